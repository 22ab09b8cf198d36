"""GCN candidate-route scorer training on the GPU (csrc/gcn_train.hip).

* the HIP backward's flat gradient matches autograd of the fp32 model on the same loss, per
  parameter group, relative to the group's gradient norm;
* training on the learned edge times makes the scorer rank candidate routes (shortest path +
  via-node detours, from the batched A*) like their true travel times: Spearman >= 0.8 on
  held-out trips, well above the random-init floor;
* data parallel by node rows (2 rank processes on one GPU): ranks end bit-identical and match
  single-rank training.
Reference: the reference takes one ORS route per trip with no alternatives (RO/Flaskr/utils.py:147-165)."""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _graph(n=6000, seed=3):
    from routest_amd.data.graph import synth_road_graph
    from routest_amd.routing.graph import edge_costs
    from routest_amd.serve.eta_service import default_model
    g = synth_road_graph(n, seed=seed)
    cost = edge_costs(g, default_model(hidden=64, steps=80), device=torch.device("cuda", 0))
    return g, cost


def test_hip_gradient_matches_autograd():
    from routest_amd.models.gcn import GcnScorer
    from routest_amd.models.gcn_train import (PARAM_SHAPES, GcnTrainerHip, GcnTrainerTorch, check_symmetric,
                                              node_delay_targets)
    g, cost = _graph()
    assert check_symmetric(g)
    t = node_delay_targets(g, cost)
    ref = GcnTrainerTorch(GcnScorer(seed=1), g, t).grad()
    hip = GcnTrainerHip(GcnScorer(seed=1), g, t, "cuda:0").grad().cpu()
    o = 0
    for name, shp in PARAM_SHAPES:
        k = int(np.prod(shp)) if shp else 1
        a, b = hip[o:o + k], ref[o:o + k]
        rel = float((a - b).norm() / (b.norm() + 1e-12))
        assert rel < 3e-2, (name, rel)       # bf16 operands (as the forward), fp32 accumulation
        o += k


def test_training_ranks_alternatives_like_true_times():
    from routest_amd.models.gcn import GcnScorer, GcnScorerHip
    from routest_amd.models.gcn_train import (candidate_routes, evaluate_ranking, node_delay_targets,
                                              score_with_delays, train, via_alternatives)
    from routest_amd.routing.graph import BatchedAstar
    g, cost = _graph(20000, seed=4)
    model, info = train(g, cost, steps=300, lr=5e-3, device="cuda:0", log_every=50)
    h = info["history"]
    assert h[-1]["mse"] < 0.25 * h[0]["mse"], h
    astar = BatchedAstar(g, cost, torch.device("cuda", 0), slots=2048)
    trips = via_alternatives(g, 150, k=4, seed=99)           # held-out trips
    routes, secs = candidate_routes(trips, astar.paths)
    dev = torch.device("cuda", 0)

    def delays(m):
        hip = GcnScorerHip(m, g, dev)
        return hip.node_delays().cpu().numpy()
    trained = evaluate_ranking(routes, secs, score_with_delays(g, delays(model), routes))
    floor = evaluate_ranking(routes, secs, score_with_delays(g, delays(GcnScorer(seed=0)), routes))
    assert trained["spearman_within_trip_mean"] >= 0.8, (trained, floor)
    assert trained["spearman_all_routes"] >= 0.95, trained
    assert trained["spearman_within_trip_mean"] > floor["spearman_within_trip_mean"] + 0.1, (trained, floor)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _dp_worker(rank, world, port, out):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from routest_amd.models.gcn import GcnScorer
    from routest_amd.models.gcn_train import GcnTrainerHip, node_delay_targets
    from routest_amd.data.graph import synth_road_graph
    g = synth_road_graph(6000, seed=3)
    cost = (g.length_m / 8.0).astype(np.float32)
    t = node_delay_targets(g, cost)

    class _CpuComm:                        # gloo on host copies (RCCL refuses two ranks per GPU)
        def all_reduce(self, x):
            y = x.cpu()
            dist.all_reduce(y)
            x.copy_(y)
    tr = GcnTrainerHip(GcnScorer(seed=2), g, t, "cuda:0", rank=rank, world=world, comm=_CpuComm())
    for _ in range(20):
        tr.step()
    torch.save(tr.P.detach().cpu(), os.path.join(out, f"p{rank}.pt"))
    dist.destroy_process_group()


def test_data_parallel_rows_match_single_rank(tmp_path):
    import torch.multiprocessing as mp
    from routest_amd.data.graph import synth_road_graph
    from routest_amd.models.gcn import GcnScorer
    from routest_amd.models.gcn_train import GcnTrainerHip, node_delay_targets
    mp.spawn(_dp_worker, args=(2, _port(), str(tmp_path)), nprocs=2, join=True)
    p0 = torch.load(tmp_path / "p0.pt")
    p1 = torch.load(tmp_path / "p1.pt")
    assert torch.equal(p0, p1)
    g = synth_road_graph(6000, seed=3)
    t = node_delay_targets(g, (g.length_m / 8.0).astype(np.float32))
    tr = GcnTrainerHip(GcnScorer(seed=2), g, t, "cuda:0")
    for _ in range(20):
        tr.step()
    ps = tr.P.detach().cpu()
    assert float((ps - p0).abs().max()) < 1e-3 * float(ps.abs().max())
