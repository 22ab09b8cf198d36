"""DeviceComm's one-shot set-up is ONE decision for all ranks (parallel/comm.py), checked on CPU with
gloo and a stand-in for the native communicator whose ``comm_open_peers`` fails like
``hipIpcOpenMemHandle`` does on the faulted rank.  The GPU version of the same scenario, with the
real HIP call failing, is tests/test_multirank_gpu.py::test_ipc_open_failure_on_one_rank_is_one_decision_for_all.
"""
import contextlib
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _FakeC:
    """The native calls DeviceComm makes during set-up; opening fails on corrupted (all-zero) handles."""

    def __init__(self, rank):
        self.rank = rank

    def comm_create(self, uid, rank, world, device, oneshot_bytes, use_rccl):
        return 7

    def comm_ipc_handles(self, h):
        return bytes([self.rank + 1]) * 128

    def comm_open_peers(self, h, handles):
        if any(not any(x) for x in handles):
            raise RuntimeError("hipIpcOpenMemHandle: invalid argument")

    def comm_error(self, h):
        return 0

    def comm_destroy(self, h):
        pass


def _worker(rank, world, port, fault, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                          ROUTEST_FAULT=fault)
        os.environ.pop("LOCAL_WORLD_SIZE", None)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import routest_amd.parallel.comm as cm
        cm.native = lambda required=True: _FakeC(rank)
        torch.cuda.device = lambda d: contextlib.nullcontext()
        c = cm.DeviceComm(torch.device("cuda", 0), use_rccl=False, oneshot_bytes=1 << 20)
        v = torch.full((64,), float(rank + 1))
        algo = c.pick(v)
        if algo == "pg":
            c.all_reduce(v)
        out = torch.empty(world * 4)
        if algo == "pg":
            c.all_gather(torch.full((4,), float(rank)), out)
        q.put((rank, c.oneshot, algo, c.oneshot_error, v.tolist(), out.tolist()))
        dist.barrier()
        dist.destroy_process_group()
    except BaseException as e:  # noqa: BLE001
        q.put((rank, "error", repr(e), None, None, None))


def _run(world, fault):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, fault, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    try:
        for _ in ps:
            r = q.get(timeout=120)
            res[r[0]] = r[1:]
    finally:
        for p in ps:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    return [res[r] for r in range(world)]


@pytest.mark.parametrize("world,bad", [(2, 1), (4, 2)])
def test_one_rank_ipc_failure_disables_oneshot_everywhere(world, bad):
    res = _run(world, f"ipc_open@{bad}")
    assert all(r[0] is False for r in res), res
    assert all(r[1] == "pg" for r in res)                    # same fallback on every rank
    assert "hipIpcOpenMemHandle" in res[bad][2]
    assert all(f"rank(s) [{bad}]" in res[r][2] for r in range(world) if r != bad)
    tot = float(world * (world + 1) // 2)
    assert all(r[3] == [tot] * 64 for r in res)              # the fallback all-reduce is correct
    want = [float(r) for r in range(world) for _ in range(4)]
    assert all(r[4] == want for r in res)


def test_no_fault_keeps_oneshot_on_every_rank():
    res = _run(2, "")
    assert all(r[0] is True and r[1] == "oneshot" and r[2] is None for r in res), res
