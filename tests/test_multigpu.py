"""One rank per GPU over RCCL — the node-level paths, run when >= 2 GPUs are
visible (skipped on the 1-GPU box by the ``multigpu`` marker).  ``ROUTEST_TEST_SHARE_GPU=1``
rehearses the same workers on ONE GPU (every rank on GPU 0, gloo bootstrap instead of RCCL, the
one-shot data path unchanged) so the test logic itself is exercised where only one GPU exists.

* RCCL all-reduce / all-gather through the native communicator (own ``ncclComm``) and the
  one-shot xGMI all-reduce: exact sums of small integers, both parities
* GCN row partition over RCCL and over the one-shot all-gather == replicate, bit for bit
* fused DP trainer with the one-shot all-reduce: identical parameters on every rank
* ``bench.py --gpus N`` launches N ranks itself and reports the whole-node line
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

from routest_amd.utils import bench_schema as S

SHARE = os.environ.get("ROUTEST_TEST_SHARE_GPU", "0") == "1"
pytestmark = [pytest.mark.gpu] + ([] if SHARE else [pytest.mark.multigpu])
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _world() -> int:
    if SHARE:
        return 2
    return min(8, torch.cuda.device_count())


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _entry(fn, rank, world, port, q, args):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                          WORLD_SIZE=str(world), LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world))
        import torch.distributed as dist
        dev = torch.device("cuda", 0 if SHARE else rank)
        torch.cuda.set_device(dev)
        if SHARE:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        else:
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        res = fn(rank, world, dev, *args)
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


# ----------------------------------------------------------------------------- collectives
def _coll_worker(rank, world, dev):
    from routest_amd.parallel.comm import DeviceComm
    c = DeviceComm(dev, use_rccl=not SHARE, oneshot_bytes=8 << 20)
    assert c.oneshot
    tri = float(world * (world + 1) // 2)
    algos = ["oneshot"] + ([] if SHARE else ["rccl"])
    for it in range(4):                                     # both one-shot parities
        for algo in algos:
            n = 74_000 if it % 2 == 0 else 1_075_000        # the H=256 and H=1024 buckets
            v = torch.full((n,), float(rank + 1 + it), device=dev)
            c.all_reduce(v, algo)
            torch.cuda.synchronize()
            c.check()
            assert torch.equal(v.cpu(), torch.full((n,), tri + world * it)), (algo, it)
    shard = torch.arange(4096, dtype=torch.float32, device=dev) + 10_000 * rank
    out = torch.empty(world * 4096, device=dev)
    for algo in algos:
        out.zero_()
        c.all_gather(shard, out, algo)
        torch.cuda.synchronize()
        ref = torch.cat([torch.arange(4096, dtype=torch.float32) + 10_000 * r for r in range(world)])
        assert torch.equal(out.cpu(), ref), algo
    c.close()
    return True


def test_native_collectives_one_rank_per_gpu():
    _spawn(_coll_worker, _world())


# ----------------------------------------------------------------------------- GCN partition
def _gcn_worker(rank, world, dev, n):
    from routest_amd.data.graph import synth_road_graph
    from routest_amd.models.gcn import GcnScorer, GcnScorerHip
    from routest_amd.parallel.comm import DeviceComm
    g = synth_road_graph(n, seed=3)
    m = GcnScorer(seed=4)
    rep = GcnScorerHip(m, g, dev).node_delays().clone()
    comm = DeviceComm(dev, use_rccl=False, oneshot_bytes=8 << 20)
    out = []
    for c in ([comm] if SHARE else [None, comm]):       # RCCL (ProcessGroup) needs one GPU per rank
        part = GcnScorerHip(m, g, dev, mode="partition", rank=rank, world=world, comm=c)
        for _ in range(2):                              # the second step uses the other parity
            out.append(torch.equal(part.node_delays(), rep))
    torch.cuda.synchronize()
    comm.check()
    comm.close()
    return out


def test_gcn_partition_equals_replicate_one_rank_per_gpu():
    for res in _spawn(_gcn_worker, _world(), 20_003):
        assert all(res), res


# ----------------------------------------------------------------------------- DP trainer
def _dp_worker(rank, world, dev, steps):
    from routest_amd.data.synth import synth_records, synth_trips
    from routest_amd.models.mlp3 import EtaMLP
    from routest_amd.ops.eta_mlp import records_to_tensor
    from routest_amd.parallel.comm import DeviceComm
    from routest_amd.train.fused import FusedMlp3Trainer
    torch.manual_seed(0)
    m = EtaMLP(256)
    xs, ys = synth_trips(16384, 5)
    m.fit_normalization(xs, ys)
    B = 8192
    rec, y = synth_records(B, 100 + rank)
    comm = DeviceComm(dev, use_rccl=False)
    tr = FusedMlp3Trainer(m, dev, B, B * world, lr=1e-3, comm=comm)
    rt = records_to_tensor(rec).to(dev)
    yn = tr.normalize_targets(torch.from_numpy(y).to(dev))
    for _ in range(steps):
        tr.step(rt, yn)
    torch.cuda.synchronize()
    comm.check()
    P = tr.P.cpu().numpy().copy()
    comm.close()
    return P


def test_fused_trainer_oneshot_identical_params_one_rank_per_gpu():
    Ps = _spawn(_dp_worker, _world(), 5)
    assert np.isfinite(Ps[0]).all()
    for P in Ps[1:]:
        assert np.array_equal(P, Ps[0]), "ranks diverged"


# ----------------------------------------------------------------------------- bench.py
def test_bench_launches_all_gpus():
    n = _world()
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    if SHARE:
        env["ROUTEST_BENCH_SHARE_GPU"] = "1"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--steps", "3",
                        "--warmup", "1", "--batch", "1048576", "--p50", "0", "--rec16-steps", "2",
                        "--route-requests", "2000", "--route-steps", "1"],
                       capture_output=True, text=True, timeout=400, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == n and d["finite"] is True and d["shared_gpu"] is SHARE
    assert d["config"]["global_batch"] == n * 1048576
    # every section ran and carries the schema's keys (routest_amd/utils/bench_schema.py)
    assert d["schema_problems"] == [], d["schema_problems"]
    os_ = d["dp_training_oneshot"]
    assert os_ and os_.get("params_identical_across_ranks") is True, os_
    if not SHARE:
        assert d["collectives"] and "error" not in d["collectives"][0]
    # the GCN partition over the process group (RCCL; gloo via host memory when rehearsing on one
    # GPU) and over the native one-shot all-gather
    gcn = d["gcn"]
    assert set(S.GCN_MODES_N) | {S.GCN_MODE_ONESHOT} <= set(gcn["modes"]), gcn
    for m in gcn["modes"]:
        assert gcn[m]["ms_per_step"] > 0, (m, gcn)
    # the route section: each rank its share of the requests, reductions over every rank
    ro = d["route_optimizer"]
    assert ro["ranks"] == n and ro["requests_per_step"] == 2000 // n * n, ro
    assert ro[S.ROUTE_UNFOUND] == 0 and ro["requests_per_s"] > 0, ro
