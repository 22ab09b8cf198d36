"""Stress the native one-shot collectives (csrc/comm.hip): W ranks sharing GPU 0 (gloo bootstrap),
N iterations of mixed all-reduce / all-gather / broadcast with exact integer-valued data, checked
every iteration; the fused stage+signal kernel's block tickets and both epoch parities get many
thousand rounds.  Usage: python tools/stress_oneshot.py [world] [iters]"""
import os
import socket
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def worker(rank, world, port, iters, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                          WORLD_SIZE=str(world))
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        from routest_amd.parallel.comm import DeviceComm
        c = DeviceComm(torch.device("cuda", 0), use_rccl=False, oneshot_bytes=2 << 20)
        tri = world * (world + 1) // 2
        bad = 0
        for it in range(iters):
            n = (1 + (it * 7919) % 4096) * 4                 # varying sizes -> varying grids
            v = torch.full((n,), float(rank + 1 + (it % 5)), device="cuda")
            c.all_reduce(v, "oneshot")
            if it % 3 == 0:
                sh = torch.full((1000 + 4 * (it % 7),), float(rank * 100 + it % 11), device="cuda")
                out = torch.empty(sh.numel() * world, device="cuda")
                c.all_gather(sh, out, "oneshot")
            if it % 5 == 0:
                b = torch.full((2048,), float(rank), device="cuda")
                c.broadcast(b, it % world, "oneshot")
            if it % 50 == 0 or it == iters - 1:
                torch.cuda.synchronize()
                c.check()
                ok = torch.equal(v, torch.full_like(v, float(tri + world * (it % 5))))
                if it % 3 == 0:
                    ref = torch.cat([torch.full((sh.numel(),), float(r * 100 + it % 11), device="cuda")
                                     for r in range(world)])
                    ok = ok and torch.equal(out, ref)
                if it % 5 == 0:
                    ok = ok and torch.equal(b, torch.full_like(b, float(it % world)))
                bad += 0 if ok else 1
        torch.cuda.synchronize()
        c.check()
        c.close()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, bad))
    except BaseException as e:  # noqa: BLE001
        q.put((rank, repr(e)))


def main():
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 3000
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, world, port, iters, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=600) for _ in ps)
    for p in ps:
        p.join(timeout=30)
    print({"world": world, "iters": iters, "checks_failed_per_rank": res}, flush=True)
    return 0 if all(v == 0 for v in res.values()) else 1


if __name__ == "__main__":
    sys.exit(main())
