"""Native collectives (csrc/comm.hip): own RCCL communicator + one-shot IPC all-reduce.

The one-shot path is exercised with 2 ranks sharing GPU 0 (IPC handles between two processes on
one device): same code path as 8 ranks over xGMI, minus the remote links.  Each rank checks the
exact sum (fixed rank order), both buffer parities, and replay of a captured HIP graph."""
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_comm_world1_rccl():
    from routest_amd.parallel.comm import DeviceComm
    c = DeviceComm(torch.device("cuda", 0), rank=0, world=1, use_rccl=True)
    try:
        x = torch.arange(1024, dtype=torch.float32, device="cuda")
        y = x.clone()
        c.all_reduce(y)
        out = torch.empty_like(x)
        c.all_gather(x, out)
        c.C.comm_all_reduce(c.h, y, 0)          # direct RCCL call with one rank
        rs = torch.empty_like(x)
        c.reduce_scatter(x, rs)
        torch.cuda.synchronize()
        assert torch.equal(y, x) and torch.equal(out, x) and torch.equal(rs, x)
        assert c.C.rccl_version() > 0
    finally:
        c.close()


def _worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        from routest_amd.parallel.comm import DeviceComm
        c = DeviceComm(torch.device("cuda", 0), use_rccl=False, oneshot_bytes=1 << 20)
        assert c.oneshot
        n = 74000                                   # the H=256 gradient bucket
        g = torch.Generator().manual_seed(0)
        base = [torch.randn(n, generator=g) for _ in range(world)]
        for it in range(5):                         # both parities, several epochs
            t = (base[rank] * (it + 1)).cuda()
            c.all_reduce(t, "oneshot")
            torch.cuda.synchronize()
            c.check()
            ref = base[0] * (it + 1)
            for r in range(1, world):
                ref = ref + base[r] * (it + 1)
            assert torch.equal(t.cpu(), ref), f"eager iter {it}"
        # graph capture: stage src -> x, all-reduce x
        src = torch.empty(n, device="cuda")
        x = torch.empty(n, device="cuda")
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            x.copy_(src)
        torch.cuda.synchronize()
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            x.copy_(src)
            c.all_reduce(x, "oneshot")
        for it in range(4):
            src.copy_((base[rank] - it).cuda())
            gr.replay()
            torch.cuda.synchronize()
            c.check()
            ref = base[0] - it
            for r in range(1, world):
                ref = ref + (base[r] - it)
            assert torch.equal(x.cpu(), ref), f"graph replay {it}"
        dist.barrier()
        c.close()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except BaseException as e:  # noqa: BLE001
        q.put((rank, repr(e)))


def test_oneshot_allreduce_two_ranks_one_gpu():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in procs:
            r, msg = q.get(timeout=240)
            res[r] = msg
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    assert res == {0: "ok", 1: "ok"}, res
