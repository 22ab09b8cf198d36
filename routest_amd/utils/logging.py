"""stdlib logging with an optional JSON formatter (the reference only print()s,
``RO/Flaskr/routes.py:125,158,179``)."""
from __future__ import annotations

import json
import logging
import sys
import time

_CONFIGURED = False


class JsonFormatter(logging.Formatter):
    def format(self, record: logging.LogRecord) -> str:
        d = {"ts": round(time.time(), 6), "level": record.levelname, "logger": record.name,
             "msg": record.getMessage()}
        extra = getattr(record, "extra_fields", None)
        if isinstance(extra, dict):
            d.update(extra)
        if record.exc_info:
            d["exc"] = self.formatException(record.exc_info)
        return json.dumps(d, default=str)


def setup_logging(json_logs: bool = False, level: int = logging.INFO) -> None:
    global _CONFIGURED
    if _CONFIGURED:
        return
    h = logging.StreamHandler(sys.stderr)
    h.setFormatter(JsonFormatter() if json_logs else
                   logging.Formatter("%(asctime)s %(levelname)s %(name)s: %(message)s"))
    root = logging.getLogger("routest_amd")
    root.addHandler(h)
    root.setLevel(level)
    root.propagate = False
    _CONFIGURED = True


def get_logger(name: str) -> logging.Logger:
    return logging.getLogger("routest_amd." + name)
