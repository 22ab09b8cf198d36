"""K9 batched A* vs scipy Dijkstra on the synthetic road graph with MLP edge costs."""
import numpy as np
import pytest
import torch

from routest_amd.data.graph import synth_road_graph, synth_route_queries
from routest_amd.routing.graph import BatchedAstar, dijkstra_ref, edge_costs
from routest_amd.serve.eta_service import default_model

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def graph_and_cost():
    g = synth_road_graph(100_000, seed=5)
    m = default_model(hidden=64, steps=50)
    cost_gpu = edge_costs(g, m, device="cuda:0")
    cost_cpu = edge_costs(g, m, device=None)
    return g, cost_gpu, cost_cpu


def test_edge_costs_kernel_vs_cpu(graph_and_cost):
    g, cg, cc = graph_and_cost
    assert (cg > 0).all()
    np.testing.assert_allclose(cg, cc, rtol=1e-2, atol=0.05)


def test_astar_optimal_costs_and_valid_paths(graph_and_cost):
    g, cost, _ = graph_and_cost
    src, dst = synth_route_queries(g, 2000, seed=1)
    a = BatchedAstar(g, cost, "cuda:0", slots=1024, cap=65536)
    c, n, st, p = a.run(src, dst)
    c, n, st, p = c.cpu().numpy(), n.cpu().numpy(), st.cpu().numpy(), p.cpu().numpy()
    assert (st == 0).mean() > 0.99
    ref = dijkstra_ref(g, cost, src, dst)
    ok = st == 0
    np.testing.assert_allclose(c[ok], ref[ok], rtol=1e-4)
    # each path is a real edge sequence from src to dst whose cost sums to the reported cost
    for i in np.where(ok)[0][:200]:
        path = p[i, :n[i]]
        assert path[0] == src[i] and path[-1] == dst[i]
        tot = 0.0
        for u, v in zip(path[:-1], path[1:]):
            nb = g.indices[g.indptr[u]:g.indptr[u + 1]]
            k = np.where(nb == v)[0]
            assert len(k) == 1
            tot += cost[g.indptr[u] + k[0]]
        assert abs(tot - c[i]) <= 1e-3 * max(1.0, c[i])
    # workspace was restored: a second batch gives identical answers
    c2 = a.run(src, dst)[0].cpu().numpy()
    assert np.array_equal(c, c2)
