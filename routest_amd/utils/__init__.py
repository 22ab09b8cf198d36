from .timeutil import parse_iso, coerce_pickup, wallclock_seconds  # noqa: F401
from .logging import get_logger, setup_logging  # noqa: F401
