"""One rank per GPU, started by the benchmark itself (SURVEY §2.9 "torchrun --nproc-per-node").

``ensure_ranks(gpus)`` is called first thing by every multi-GPU entry point (``bench.py``,
``bench/*_bench.py``):

* WORLD_SIZE set (launched by ``torch.distributed.run`` / torchrun): it must equal ``gpus``,
  otherwise exit 2 — a run can never silently measure fewer GPUs than asked for.
* WORLD_SIZE unset and ``gpus > 1``: start ``python -m torch.distributed.run --nproc-per-node
  gpus`` on the same script and arguments as a CHILD process, wait, and exit with its code.  This
  happens before anything touches the GPU in the parent (``torch.cuda.device_count`` does not
  initialise HIP) and never ``exec``s.  Fewer visible GPUs than ``gpus`` exits 2.

``ROUTEST_BENCH_SHARE_GPU=1`` is the 1-GPU-box rehearsal: all ranks on GPU 0 with a gloo
rendezvous (RCCL refuses two ranks on one device); results carry ``shared_gpu: true``.
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys
from typing import List, Optional

SHARE_ENV = "ROUTEST_BENCH_SHARE_GPU"


def share_gpu() -> bool:
    return os.environ.get(SHARE_ENV) == "1"


def free_port() -> int:
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_child(gpus: int, script: str, argv: List[str]) -> int:
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={free_port()}", os.path.abspath(script)] + argv
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "4")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def ensure_ranks(gpus: int, script: Optional[str] = None, argv: Optional[List[str]] = None) -> int:
    """Returns the world size this process runs in (== gpus), or exits (see module doc)."""
    if gpus < 1:
        print(f"{script or sys.argv[0]}: --gpus must be >= 1", file=sys.stderr)
        sys.exit(2)
    script = script or sys.argv[0]
    if "WORLD_SIZE" not in os.environ:
        if gpus == 1:
            return 1
        if not share_gpu():
            import torch
            n_vis = torch.cuda.device_count()
            if gpus > n_vis:
                print(f"{os.path.basename(script)}: --gpus {gpus} but only {n_vis} GPU(s) visible",
                      file=sys.stderr)
                sys.exit(2)
        sys.exit(launch_child(gpus, script, list(sys.argv[1:] if argv is None else argv)))
    world = int(os.environ["WORLD_SIZE"])
    if world != gpus:
        print(f"{os.path.basename(script)}: WORLD_SIZE={world} but --gpus {gpus}", file=sys.stderr)
        sys.exit(2)
    if not share_gpu():
        import torch
        lr = int(os.environ.get("LOCAL_RANK", "0"))
        if lr >= torch.cuda.device_count():
            print(f"{os.path.basename(script)}: LOCAL_RANK {lr} has no GPU "
                  f"({torch.cuda.device_count()} visible)", file=sys.stderr)
            sys.exit(2)
    return world
