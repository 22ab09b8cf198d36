"""GCN scorer training, CPU reference (models/gcn_train.py): per-node targets from edge times, the
autograd trainer, via-node alternatives and the ranking metric.  The HIP kernels are checked
against this in tests/test_gcn_train_gpu.py."""
import numpy as np
import pytest


def _setup(n=2500, seed=5):
    from routest_amd.data.graph import synth_road_graph
    from routest_amd.routing.graph import GraphProvider
    g = synth_road_graph(n, seed=seed)
    rng = np.random.default_rng(seed)
    # edge times: class speed x a smooth congestion field (what the scorer has to learn)
    mid = np.array([g.lat.mean(), g.lon.mean()])
    src = np.repeat(np.arange(g.num_nodes), np.diff(g.indptr))
    cong = 1.0 + 1.5 * np.exp(-(((g.lat[src] - mid[0]) / 0.08) ** 2 + ((g.lon[src] - mid[1]) / 0.05) ** 2))
    speed = np.array([8.3, 12.5, 16.7, 22.2])[g.road_class]
    cost = (g.length_m / speed * cong * (1 + 0.05 * rng.standard_normal(len(src)))).astype(np.float32)
    return g, np.maximum(cost, g.length_m / 36.0).astype(np.float32), GraphProvider(g, cost, device=None)


def test_targets_and_symmetry():
    from routest_amd.models.gcn_train import V_REF, check_symmetric, node_delay_targets
    g, cost, _ = _setup()
    assert check_symmetric(g)
    t = node_delay_targets(g, cost)
    assert t.shape == (g.num_nodes,) and np.all(t > 0.5)
    # a node's target times its out-edges' great-circle length ~ V_REF x their seconds
    v = 100
    e0, e1 = g.indptr[v], g.indptr[v + 1]
    want = np.mean(cost[e0:e1] * V_REF / (g.length_m[e0:e1] / 1.15))
    assert abs(t[v] - want) < 1e-3 * want


def test_cpu_training_improves_ranking():
    from routest_amd.models.gcn import GcnScorer
    from routest_amd.models.gcn_train import (candidate_routes, evaluate_ranking, score_with_delays, train,
                                              via_alternatives)
    import torch
    g, cost, prov = _setup()
    model, info = train(g, cost, steps=150, lr=1e-2, log_every=50)
    assert info["history"][-1]["mse"] < 0.5 * info["history"][0]["mse"]
    trips = via_alternatives(g, 30, k=4, seed=7, min_km=2.0, max_km=12.0)
    assert len(trips) >= 20
    routes, secs = candidate_routes(trips, lambda s, t: prov._shortest(list(zip(s, t))))
    with torch.no_grad():
        A, X = GcnScorer.adjacency(g), torch.from_numpy(g.features)
        d_tr = model(A, X).numpy()
        d_0 = GcnScorer(seed=0)(A, X).numpy()
    tr = evaluate_ranking(routes, secs, score_with_delays(g, d_tr, routes))
    fl = evaluate_ranking(routes, secs, score_with_delays(g, d_0, routes))
    assert tr["spearman_within_trip_mean"] > fl["spearman_within_trip_mean"], (tr, fl)
    assert tr["spearman_all_routes"] > 0.9, tr
