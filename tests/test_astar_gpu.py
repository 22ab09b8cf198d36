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


@pytest.mark.parametrize("reorder", ["0", "1"])
def test_astar_optimal_costs_and_valid_paths(graph_and_cost, monkeypatch, reorder):
    """reorder=1: the searches run on the Morton-renumbered graph; paths come back in caller ids."""
    g, cost, _ = graph_and_cost
    src, dst = synth_route_queries(g, 2000, seed=1)
    monkeypatch.setenv("ROUTEST_ASTAR_REORDER", reorder)
    a = BatchedAstar(g, cost, "cuda:0", slots=1024)
    c, n, st, p = a.run(src, dst)
    c, n, st, p = c.cpu().numpy(), n.cpu().numpy(), st.cpu().numpy(), p.cpu().numpy()
    ref = dijkstra_ref(g, cost, src, dst)
    assert np.isfinite(ref).all()            # every query is connected on this graph ...
    assert (st == 0).all(), np.unique(st, return_counts=True)    # ... and every search finds it
    assert a.last_fallbacks == 0             # ... on the GPU (no host fallback involved)
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


@pytest.mark.parametrize("lane_pops,delta", [(0, 60.0), (40, 60.0), (40, 5.0), (40, 600.0)])
def test_wave_tail_stage_exact(graph_and_cost, monkeypatch, lane_pops, delta):
    """Searches that exhaust the lane budget finish in the one-wave-per-query stage with the same
    optimal costs (vs scipy Dijkstra) and valid paths; lane_pops=0 sends every query there."""
    g, cost, _ = graph_and_cost
    src, dst = synth_route_queries(g, 600, seed=2)
    src[:3] = dst[:3]                                   # s == t queries too
    monkeypatch.setenv("ROUTEST_ASTAR_LANE_POPS", str(lane_pops if lane_pops else 1))
    monkeypatch.setenv("ROUTEST_ASTAR_DELTA", str(delta))
    a = BatchedAstar(g, cost, "cuda:0", slots=1024)
    c, n, st, p = a.run(src, dst)
    assert a.last_tail > 300                            # most queries went through the wave stage
    c, n, st, p = c.cpu().numpy(), n.cpu().numpy(), st.cpu().numpy(), p.cpu().numpy()
    assert (st == 0).all()
    ref = dijkstra_ref(g, cost, src, dst)
    np.testing.assert_allclose(c, ref, rtol=1e-4, atol=1e-3)
    for i in range(0, len(src), 7):
        path = p[i, :n[i]]
        assert path[0] == src[i] and path[-1] == dst[i]
        tot = 0.0
        for u, v in zip(path[:-1], path[1:]):
            nb = g.indices[g.indptr[u]:g.indptr[u + 1]]
            k = np.where(nb == v)[0]
            assert len(k) == 1
            tot += cost[g.indptr[u] + k[0]]
        assert abs(tot - c[i]) <= 1e-3 * max(1.0, c[i])
    c2 = a.run(src, dst)[0].cpu().numpy()                 # workspace restored by both stages
    assert np.array_equal(c, c2)


def test_small_lists_grow_into_the_arena(graph_and_cost):
    """cap 128 (64-entry f-band lists, 256-entry tables): the wave tier moves its lists and tables
    into arena buffers as the searches grow, so nothing overflows to the big tier or the host."""
    g, cost, _ = graph_and_cost
    src, dst = synth_route_queries(g, 300, seed=3)
    a = BatchedAstar(g, cost, "cuda:0", slots=512, cap=128)
    c, n, st, p = a.run(src, dst)
    assert a.last_escalated == 0 and a.last_fallbacks == 0, a.last_stats
    assert (st.cpu().numpy() == 0).all()
    np.testing.assert_allclose(c.cpu().numpy(), dijkstra_ref(g, cost, src, dst), rtol=1e-4)
    assert bool((a.arena == -1).all())                   # lists and tables restored to all-ones


def test_overflowed_searches_escalate_to_the_big_tier(graph_and_cost):
    """Without the arena, wave-tier lists far too small (cap 128) overflow (status 2) and the
    searches are rerun in the big tier, whose tables hold every node — still on the GPU, at the
    optimal cost."""
    g, cost, _ = graph_and_cost
    src, dst = synth_route_queries(g, 300, seed=3)
    a = BatchedAstar(g, cost, "cuda:0", slots=512, cap=128, arena_gb=0)
    c, n, st, p = a.run(src, dst)
    assert a.last_escalated > 100 and a.last_fallbacks == 0, a.last_stats
    c, n, st, p = c.cpu().numpy(), n.cpu().numpy(), st.cpu().numpy(), p.cpu().numpy()
    assert (st == 0).all(), np.unique(st, return_counts=True)
    np.testing.assert_allclose(c, dijkstra_ref(g, cost, src, dst), rtol=1e-4)
    for i in range(0, 300, 37):
        assert p[i, 0] == src[i] and p[i, n[i] - 1] == dst[i]
    c2 = a.run(src, dst)[0].cpu().numpy()               # every tier restored its tables
    assert np.array_equal(c, c2)


def test_arena_overflows_are_retried_in_chunks(graph_and_cost):
    """A growth arena far too small for one launch's searches (2 MB for 300 concurrent searches):
    the searches that overflowed are rerun in the wave tier a chunk at a time (each chunk gets the
    whole, reset arena) before anything reaches the big tier — optimal costs, arena restored."""
    g, cost, _ = graph_and_cost
    src, dst = synth_route_queries(g, 300, seed=3)
    a = BatchedAstar(g, cost, "cuda:0", slots=512, cap=128, arena_gb=0.002)
    c, n, st, p = a.run(src, dst)
    assert a.last_stats["retried"] > 0 and a.last_fallbacks == 0, a.last_stats
    assert a.last_escalated <= a.last_stats["retried"]
    assert (st.cpu().numpy() == 0).all()
    np.testing.assert_allclose(c.cpu().numpy(), dijkstra_ref(g, cost, src, dst), rtol=1e-4)
    assert bool((a.arena == -1).all())


def test_overflowed_searches_finish_exactly_on_host(graph_and_cost):
    """Without an arena or a big tier the overflowed searches are finished by the exact host
    fallback."""
    g, cost, _ = graph_and_cost
    src, dst = synth_route_queries(g, 300, seed=3)
    a = BatchedAstar(g, cost, "cuda:0", slots=512, cap=128, big_slots=0, arena_gb=0)
    c, n, st, p = a.run(src, dst)
    assert a.last_fallbacks > 0
    c, n, st, p = c.cpu().numpy(), n.cpu().numpy(), st.cpu().numpy(), p.cpu().numpy()
    assert (st == 0).all(), np.unique(st, return_counts=True)
    np.testing.assert_allclose(c, dijkstra_ref(g, cost, src, dst), rtol=1e-4)
    for i in range(0, 300, 37):
        assert p[i, 0] == src[i] and p[i, n[i] - 1] == dst[i]


def test_lane_tier_overflow_continues_in_the_wave_tier(graph_and_cost, monkeypatch):
    """Big batches run the lane tier first; its small tables overflow on long legs (status 2) and
    those searches continue in the wave tier like the ones whose pop budget ran out."""
    g, cost, _ = graph_and_cost
    src, dst = synth_route_queries(g, 1500, seed=4)
    monkeypatch.setenv("ROUTEST_ASTAR_WAVE_ONLY_BELOW", "0")       # force the lane tier
    monkeypatch.setenv("ROUTEST_ASTAR_LANE_POPS", "2000")          # long budget, small tables overflow
    monkeypatch.setenv("ROUTEST_ASTAR_LANE_MAX_M", "0")            # every leg starts in the lane tier
    a = BatchedAstar(g, cost, "cuda:0", slots=1024)
    a.lane_tier = type(a.lane_tier)(1024, 64, 7, a.dev)            # 128-entry tables: overflow early
    c, n, st, p = a.run(src, dst)
    assert a.last_stats["lane"] == 1500 and a.last_tail > 500, a.last_stats
    st = st.cpu().numpy()
    assert (st == 0).all()
    np.testing.assert_allclose(c.cpu().numpy(), dijkstra_ref(g, cost, src, dst), rtol=1e-4)


def test_long_legs_skip_the_lane_tier_exactly(graph_and_cost, monkeypatch):
    """ROUTEST_ASTAR_LANE_MAX_M: legs longer than the threshold (great circle) go straight to the wave
    tier, which takes them longest first; the short ones run the lane tier from a compacted index
    list.  Every cost stays optimal and exactly the short legs ran the lane tier."""
    g, cost, _ = graph_and_cost
    src, dst = synth_route_queries(g, 1500, seed=5)
    la, lb = np.radians(g.lat[src]), np.radians(g.lat[dst])
    dl = np.radians(g.lon[dst] - g.lon[src])
    hv = np.sin(0.5 * (lb - la)) ** 2 + np.cos(la) * np.cos(lb) * np.sin(0.5 * dl) ** 2
    d = 2 * 6371000.0 * np.arcsin(np.sqrt(np.clip(hv, 0, 1)))
    thr = float(np.median(d))
    monkeypatch.setenv("ROUTEST_ASTAR_WAVE_ONLY_BELOW", "0")       # force the lane tier
    monkeypatch.setenv("ROUTEST_ASTAR_LANE_MAX_M", str(thr))
    a = BatchedAstar(g, cost, "cuda:0", slots=1024)
    c, n, st, p = a.run(src, dst)
    short = int((d <= thr * (1 - 1e-4)).sum())
    assert short <= a.last_stats["lane"] <= int((d <= thr * (1 + 1e-4)).sum()), (a.last_stats, short)
    assert a.last_stats["lane"] < 1500
    assert (st.cpu().numpy() == 0).all()
    np.testing.assert_allclose(c.cpu().numpy(), dijkstra_ref(g, cost, src, dst), rtol=1e-4)


def test_wave_tables_grow_into_the_arena_exactly(graph_and_cost, monkeypatch):
    """Wave-tier tables that start at 64 entries grow 4x at a time into the shared arena (parent
    pointers rewritten at every rehash): every search still finishes on the GPU at the optimal cost,
    and the arena is restored (a second run gives identical answers)."""
    g, cost, _ = graph_and_cost
    src, dst = synth_route_queries(g, 800, seed=6)
    monkeypatch.setenv("ROUTEST_ASTAR_WAVE_TBITS", "6")
    a = BatchedAstar(g, cost, "cuda:0", slots=1024)
    assert a.wave_tier.tbits == 6
    c, n, st, p = a.run(src, dst)
    assert a.last_escalated == 0 and a.last_fallbacks == 0, a.last_stats
    c, n, st, p = c.cpu().numpy(), n.cpu().numpy(), st.cpu().numpy(), p.cpu().numpy()
    assert (st == 0).all()
    np.testing.assert_allclose(c, dijkstra_ref(g, cost, src, dst), rtol=1e-4, atol=1e-3)
    for i in range(0, len(src), 41):
        path = p[i, :n[i]]
        assert path[0] == src[i] and path[-1] == dst[i]
        tot = 0.0
        for u, v in zip(path[:-1], path[1:]):
            nb = g.indices[g.indptr[u]:g.indptr[u + 1]]
            k = np.where(nb == v)[0]
            assert len(k) == 1
            tot += cost[g.indptr[u] + k[0]]
        assert abs(tot - c[i]) <= 1e-3 * max(1.0, c[i])
    assert bool((a.arena == -1).all())                   # every grown table restored to all-ones
    c2 = a.run(src, dst)[0].cpu().numpy()
    assert np.array_equal(c, c2)


def test_workspace_is_independent_of_graph_size(graph_and_cost):
    """Sparse per-search state: the lane and wave tiers do not grow with N (only the big tier's
    tables are sized from the graph)."""
    g, cost, _ = graph_and_cost
    a = BatchedAstar(g, cost, "cuda:0", slots=1024, big_slots=0)
    small = synth_road_graph(5_000, seed=1)
    b = BatchedAstar(small, edge_costs(small, default_model(hidden=64, steps=5), device="cuda:0"), "cuda:0",
                     slots=1024, big_slots=0)
    assert a.workspace_bytes == b.workspace_bytes


@pytest.mark.parametrize("nw", [1, 2, 4, 8])
def test_multi_wave_searches_exact(graph_and_cost, nw):
    """Every waves-per-search instantiation (the s_next reset raced with slower waves
    when NW > 1) on the three paths that use it: the main wave tier, the arena reruns and the big
    tier — optimal costs vs scipy Dijkstra, workspace restored (a second run is identical)."""
    g, cost, _ = graph_and_cost
    src, dst = synth_route_queries(g, 400, seed=11)
    ref = dijkstra_ref(g, cost, src, dst)
    for kw, key in ((dict(cap=128, arena_gb=0.002), "retried"), (dict(cap=128, arena_gb=0), "escalated"),
                    (dict(), "wave")):
        a = BatchedAstar(g, cost, "cuda:0", slots=512, **kw)
        a.wave_nw = nw
        a.retry_nw = nw
        c, n, st, p = a.run(src, dst)
        assert a.last_stats[key] > 0 and a.last_fallbacks == 0, (kw, a.last_stats)
        assert (st.cpu().numpy() == 0).all(), (kw, np.unique(st.cpu().numpy(), return_counts=True))
        np.testing.assert_allclose(c.cpu().numpy(), ref, rtol=1e-4)
        assert np.array_equal(c.cpu().numpy(), a.run(src, dst)[0].cpu().numpy())


def test_unsupported_wave_count_is_an_error(graph_and_cost):
    g, cost, _ = graph_and_cost
    a = BatchedAstar(g, cost, "cuda:0", slots=64)
    a.wave_nw = 3
    with pytest.raises(RuntimeError):
        a.run([0], [1])
