"""bench.py's JSON-line schema on the CPU (routest_amd/utils/bench_schema.py).

The GPU tests assert on keys of the line bench.py prints; those keys come from the builders here,
so a rename shows up on the CPU first.  The cross-rank reductions of the route section and the
host-staged GCN all-gather (the shared-GPU rehearsal's gloo path) run with 2 gloo ranks.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from routest_amd.utils import bench_schema as S

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _line(**over):
    d = {k: None for k in S.HEADLINE + S.SECTIONS}
    d.update(metric="m", value=1.0, n_gpus=2, finite=True, shared_gpu=False,
             config={"model": "mlp3", "global_batch": 2, "seq_len": None, "parallelism": "dp2"})
    d.update(over)
    return d


def test_complete_line_has_no_problems():
    g = S.gcn_section(100, 200, 10)
    S.gcn_mode(g, "replicate", 1.0, 10, 10)
    S.gcn_mode(g, "partition", 0.5, 10, 10)
    r = S.route_section(2000, 2, 1.0, 9000, 0, 100_000, 40.0, {"cost_ms": 1.0, "customize_ms": 30.0},
                        3.0, {"levels": 5}, 2)
    tr = S.dp_training(1e8, 0.07, 65536, 2, 200, "RCCL", 0.1)
    os_ = S.dp_training(1e8, 0.07, 65536, 2, 200, "oneshot", 0.1, comm_error=False,
                        params_identical_across_ranks=True)
    d = _line(gcn=g, route_optimizer=r, dp_training=tr, dp_training_oneshot=os_,
              dp_training_large_batch=tr)
    assert S.problems(d) == []
    assert d["route_optimizer"][S.ROUTE_UNFOUND] == 0
    assert g["modes"] == ["replicate", "partition"] and g["partition"]["ms_per_step"] == 50.0


def test_drift_and_errors_are_reported():
    r = S.route_section(10, 1, 1.0, 10, 0, 5, 1.0, {}, 0.1, {}, 1)
    del r[S.ROUTE_UNFOUND]
    d = _line(route_optimizer=r, gcn={"error": "boom"})
    del d["finite"]
    p = S.problems(d)
    assert "finite" in p and "route_optimizer.unfound_legs" in p
    assert any(x.startswith("gcn: error boom") for x in p)
    r2 = S.route_section(10, 1, 1.0, 10, 0, 5, 1.0, {}, 0.1, {}, 1)
    r2["http_f02"] = {"req_per_s": 1.0}
    assert "route_optimizer.http_f02.p99_ms" in S.problems(_line(route_optimizer=r2))


def test_bench_py_uses_the_schema():
    """bench.py builds its sections through the schema's builders and reports schema_problems."""
    src = open(os.path.join(ROOT, "bench.py")).read()
    for name in ("bench_schema.route_section", "bench_schema.gcn_section", "bench_schema.gcn_mode",
                 "bench_schema.dp_training", "bench_schema.problems", "bench_schema.reduce_route_stats"):
        assert name in src, name
    assert "astar_unfound_legs" not in open(os.path.join(ROOT, "tests", "test_multigpu.py")).read()


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        # route section: slowest rank's seconds, summed legs / unfound legs
        t, legs, unf = S.reduce_route_stats(1.5 + rank, 1000 * (rank + 1), rank, torch.device("cpu"))
        # the GCN partition's host-staged all-gather (bf16 shards of Z)
        own = torch.full((4, 2), float(rank + 1), dtype=torch.bfloat16)
        full = torch.empty(4 * world, 2, dtype=torch.bfloat16)
        dist.all_gather_into_tensor(full, own)
        q.put((rank, t, legs, unf, full.float().flatten().tolist()))
        dist.destroy_process_group()
    except BaseException as e:  # noqa: BLE001
        q.put((rank, repr(e), None, None, None))


@pytest.mark.timeout(120)
def test_route_reductions_gloo_two_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = {}
    for _ in ps:
        r, *v = q.get(timeout=100)
        res[r] = v
    for p in ps:
        p.join(timeout=20)
    for r in range(2):
        t, legs, unf, full = res[r]
        assert t == 2.5 and legs == 3000 and unf == 1, res[r]
        assert full == [1.0] * 8 + [2.0] * 8
