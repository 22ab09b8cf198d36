"""Multi-rank paths run for real on ONE GPU: 2 and 4 rank processes share GPU 0 (gloo rendezvous
for the bootstrap; the data path is the native one-shot IPC protocol of csrc/comm.hip, the same
code that runs over xGMI between 8 GPUs, minus the remote links).

* one-shot all-gather / broadcast: exact, both buffer parities, HIP-graph replay
* GCN row partition (P3/C4) through DeviceComm == replicate, bit for bit
* fused HIP trainer (P1/C1) with the one-shot gradient all-reduce: parameters bit-identical on
  every rank and equal (to fp32 summation order) to one rank training on the concatenated batch
* the micro-batcher with 2 runners (P2) answers exactly what one kernel launch answers
"""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _entry(fn, rank, world, port, q, args):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                          WORLD_SIZE=str(world))
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        res = fn(rank, world, *args)
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok", res))
    except BaseException as e:  # noqa: BLE001
        import traceback
        q.put((rank, repr(e) + "\n" + traceback.format_exc()[-1500:], None))


def _spawn(fn, world, *args, timeout=240):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_entry, args=(fn, r, world, port, q, args)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in procs:
            r, msg, val = q.get(timeout=timeout)
            res[r] = (msg, val)
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    assert {r: m for r, (m, _) in res.items()} == {r: "ok" for r in range(world)}, res
    return [res[r][1] for r in range(world)]


# ----------------------------------------------------------------------------- one-shot gather
def _gather_worker(rank, world):
    from routest_amd.parallel.comm import DeviceComm
    c = DeviceComm(torch.device("cuda", 0), use_rccl=False, oneshot_bytes=1 << 20)
    assert c.oneshot
    g = torch.Generator().manual_seed(3)
    shards = [torch.randn(4096, 32, generator=g).to(torch.bfloat16) for _ in range(world)]
    for it in range(5):                                   # both parities
        inp = (shards[rank] * (it + 1)).cuda()
        out = torch.empty(world * 4096, 32, dtype=torch.bfloat16, device="cuda")
        c.all_gather(inp, out, "oneshot")
        torch.cuda.synchronize()
        c.check()
        assert torch.equal(out.cpu(), torch.cat([s * (it + 1) for s in shards])), f"gather {it}"
        # interleave an all-reduce: the ops share the parity buffers and epoch counter
        v = torch.full((1024,), float(rank + 1), device="cuda")
        c.all_reduce(v, "oneshot")
        torch.cuda.synchronize()
        assert torch.equal(v.cpu(), torch.full((1024,), float(world * (world + 1) // 2)))
    for root in range(world):
        b = torch.full((2048,), float(rank * 10 + root), device="cuda")
        c.broadcast(b, root, "oneshot")
        torch.cuda.synchronize()
        assert torch.equal(b.cpu(), torch.full((2048,), float(root * 10 + root))), f"bcast {root}"
    # graph capture of an in-place all-gather
    full = torch.zeros(world * 1000, dtype=torch.float32, device="cuda")
    src = torch.empty(1000, device="cuda")
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        full[rank * 1000:(rank + 1) * 1000].copy_(src)
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        full[rank * 1000:(rank + 1) * 1000].copy_(src)
        c.all_gather(full[rank * 1000:(rank + 1) * 1000], full, "oneshot")
    for it in range(3):
        src.fill_(float(100 * it + rank))
        gr.replay()
        torch.cuda.synchronize()
        c.check()
        ref = torch.cat([torch.full((1000,), float(100 * it + r)) for r in range(world)])
        assert torch.equal(full.cpu(), ref), f"graph {it}"
    c.close()
    return True


@pytest.mark.parametrize("world", [2, 4])
def test_oneshot_allgather_broadcast(world):
    _spawn(_gather_worker, world)


# ----------------------------------------------------------------------------- IPC open failure
def _ipc_fail_worker(rank, world):
    # rank 1's hipIpcOpenMemHandle calls get corrupted handles (parallel/comm.py test hook), so the
    # real HIP call fails on that rank only
    os.environ["ROUTEST_FAULT"] = "ipc_open@1"
    from routest_amd.parallel.comm import DeviceComm
    c = DeviceComm(torch.device("cuda", 0), use_rccl=False, oneshot_bytes=1 << 20)
    v = torch.full((1024,), float(rank + 1), device="cuda")
    algo = c.pick(v)
    c.all_reduce(v)                                       # the agreed fallback path
    g = torch.empty(2 * 256, device="cuda")
    c.all_gather(torch.full((256,), float(rank), device="cuda"), g)
    torch.cuda.synchronize()
    out = (c.oneshot, algo, c.oneshot_error, float(v[0]), g.cpu().tolist())
    c.close()
    return out


def test_ipc_open_failure_on_one_rank_is_one_decision_for_all():
    """hipIpcOpenMemHandle fails on rank 1 only: every rank disables the one-shot path (the same
    decision everywhere — a rank that kept it would wait forever for its peer) and the collectives
    run on the fallback (RCCL when the comm has it; here, both ranks on one GPU, the gloo group)."""
    res = _spawn(_ipc_fail_worker, 2)
    assert [r[0] for r in res] == [False, False]
    assert [r[1] for r in res] == ["pg", "pg"]
    assert "hipIpcOpenMemHandle" in res[1][2], res[1][2]
    assert "rank(s) [1]" in res[0][2], res[0][2]
    assert all(r[3] == 3.0 for r in res)
    assert all(r[4] == [0.0] * 256 + [1.0] * 256 for r in res)


# ----------------------------------------------------------------------------- GCN partition
def _gcn_worker(rank, world, n):
    from routest_amd.data.graph import synth_road_graph
    from routest_amd.models.gcn import GcnScorer, GcnScorerHip
    from routest_amd.parallel.comm import DeviceComm
    g = synth_road_graph(n, seed=3)
    m = GcnScorer(seed=4)
    comm = DeviceComm(torch.device("cuda", 0), use_rccl=False, oneshot_bytes=8 << 20)
    part = GcnScorerHip(m, g, torch.device("cuda:0"), mode="partition", rank=rank, world=world, comm=comm)
    d1 = part.node_delays().clone()
    d2 = part.node_delays().clone()            # second step: the other buffer parity
    torch.cuda.synchronize()
    comm.check()
    rep = GcnScorerHip(m, g, torch.device("cuda:0")).node_delays()
    torch.cuda.synchronize()
    comm.close()
    return (torch.equal(d1, rep), torch.equal(d2, rep), d1.cpu().numpy())


@pytest.mark.parametrize("world", [2, 4])
def test_gcn_partition_device_comm_equals_replicate(world):
    res = _spawn(_gcn_worker, world, 20_003)
    for eq1, eq2, _ in res:
        assert eq1 and eq2
    for _, _, d in res[1:]:
        assert np.array_equal(d, res[0][2])


# ----------------------------------------------------------------------------- DP trainer
def _train_setup(H=256):
    from routest_amd.data.synth import synth_records, synth_trips
    from routest_amd.models.mlp3 import EtaMLP
    torch.manual_seed(0)
    m = EtaMLP(H)
    xs, ys = synth_trips(16384, 5)
    m.fit_normalization(xs, ys)
    rec, y = synth_records(2 * 8192, 77)
    return m, rec, y


def _dp_worker(rank, world, steps):
    from routest_amd.ops.eta_mlp import records_to_tensor
    from routest_amd.parallel.comm import DeviceComm
    from routest_amd.train.fused import FusedMlp3Trainer
    m, rec, y = _train_setup()
    B = len(rec) // world
    comm = DeviceComm(torch.device("cuda", 0), use_rccl=False)
    dev = torch.device("cuda:0")
    tr = FusedMlp3Trainer(m, dev, B, B * world, lr=1e-3, comm=comm)
    rt = records_to_tensor(rec[rank * B:(rank + 1) * B]).to(dev)
    yn = tr.normalize_targets(torch.from_numpy(y[rank * B:(rank + 1) * B]).to(dev))
    for _ in range(steps):
        tr.step(rt, yn)
    torch.cuda.synchronize()
    comm.check()
    P = tr.P.cpu().numpy().copy()
    comm.close()
    return P


def test_fused_trainer_oneshot_dp_two_ranks():
    from routest_amd.ops.eta_mlp import records_to_tensor
    from routest_amd.train.fused import FusedMlp3Trainer
    steps = 4
    Ps = _spawn(_dp_worker, 2, steps)
    assert np.array_equal(Ps[0], Ps[1]), "ranks diverged"
    # one rank on the concatenated batch: same math up to fp32 summation order of the gradient
    m, rec, y = _train_setup()
    dev = torch.device("cuda:0")
    tr = FusedMlp3Trainer(m, dev, len(rec), len(rec), lr=1e-3, allreduce=False)
    rt = records_to_tensor(rec).to(dev)
    yn = tr.normalize_targets(torch.from_numpy(y).to(dev))
    for _ in range(steps):
        tr.step(rt, yn)
    P1 = tr.P.cpu().numpy()
    P0 = _train_setup()[0]
    from routest_amd.train.fused import flatten_params
    P0 = flatten_params(P0).numpy()
    moved = np.abs(P1 - P0).max()
    assert moved > 1e-4                      # the steps did move the parameters
    assert np.abs(Ps[0] - P1).max() < 0.02 * moved


# ----------------------------------------------------------------------------- batcher, 2 runners
def test_micro_batcher_two_runners_same_answers():
    import concurrent.futures as cf
    from routest_amd.data.synth import synth_records
    from routest_amd.ops.eta_mlp import EtaMlpKernel, records_to_tensor
    from routest_amd.serve.batcher import GpuRunner, MicroBatcher
    m, _, _ = _train_setup()
    dev = torch.device("cuda:0")
    k = EtaMlpKernel(m, dev)
    runners = [GpuRunner(k, dev, 512), GpuRunner(k, dev, 512)]
    mb = MicroBatcher(runners, batch_max=512, timeout_us=300, inline_when_idle=False)
    try:
        rec, _ = synth_records(6000, 31)
        ref = k(records_to_tensor(rec).to(dev)).cpu().numpy()
        with cf.ThreadPoolExecutor(16) as ex:
            futs = [ex.submit(mb.predict_sync, rec[i].item()) for i in range(len(rec))]
            got = np.array([f.result(60) for f in futs], dtype=np.float32)
        np.testing.assert_array_equal(got, ref)
        assert all(h["healthy"] for h in mb.health())
    finally:
        mb.close()
