"""Native HTTP front end for the prediction endpoints (``csrc/native_server.hip``).

``POST /api/predict_eta`` and ``POST /predict`` are answered by C++ reactor threads — native JSON
packing, one zero-copy fused-kernel launch per wake-up (natural batching across connections),
CPython-exact response formatting — with no Python on the request path.  It runs next to the
FastAPI app (which keeps every other endpoint) on its own port::

    python -m routest_amd serve --synthetic-model --port 5000 --native-port 5001

The reference answers this route through Flask (``RO/Flaskr/routes.py:365-383``); this front end
exists because single-request latency is host-stack bound.
"""
from __future__ import annotations

import socket
from typing import Dict, List, Optional, Sequence

import torch

from ..ops._ext import native
from ..ops.eta_mlp import EtaMlpKernel


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class NativePredictServer:
    """``device``: one GPU index or a list — reactor threads are spread round-robin over the GPUs
    (each GPU gets its own weight copy; use ``threads >= len(devices)``)."""

    def __init__(self, model, device=0, port: int = 0, threads: int = 2, max_batch: int = 1 << 18,
                 cors_origins: Sequence[str] = ("http://localhost:3000", "http://127.0.0.1:3000"),
                 cors_vercel: bool = True, bind_any: bool = False, variant: int = -1):
        self.C = native(required=True)
        devices = [device] if isinstance(device, int) else list(device)
        threads = max(threads, len(devices))
        # one packed weight blob per GPU; the kernels keep them alive for the server's lifetime
        self.kerns = [EtaMlpKernel(model, torch.device("cuda", d), variant=variant) for d in devices]
        k0 = self.kerns[0]
        self.port = port or free_port()
        self.h: Optional[int] = self.C.native_server_start(
            self.port, threads, [k.packed.blob for k in self.kerns], k0.hidden, list(k0.packed.norm),
            variant, max_batch, list(cors_origins), cors_vercel, bind_any)

    def stats(self) -> Dict[str, int]:
        if self.h is None:
            return {}
        v = self.C.native_server_stats(self.h)
        # resident: rounds scored by the persistent kernel (csrc/persistent_serve.hip);
        # fallbacks: rounds it did not answer in time, re-scored by a normal launch;
        # wire8: launches that read 8-byte wire records (features.py RECORD8) instead of 16-byte
        names = ("requests", "predictions", "launches", "errors", "resident", "fallbacks", "wire8")
        return dict(zip(names, v))

    def close(self) -> None:
        if self.h is not None:
            self.C.native_server_stop(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False
