"""K8 GCN kernels vs the fp32 torch.sparse reference."""
import numpy as np
import pytest
import torch

from routest_amd.data.graph import synth_road_graph
from routest_amd.models.gcn import GcnScorer, GcnScorerHip, routes_to_csr, score_routes_ref

pytestmark = pytest.mark.gpu


def _random_walks(g, n, seed=0, lo=20, hi=200):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        v = int(rng.integers(0, g.num_nodes))
        path = [v]
        for _ in range(int(rng.integers(lo, hi))):
            nb = g.indices[g.indptr[v]:g.indptr[v + 1]]
            v = int(nb[rng.integers(0, len(nb))])
            path.append(v)
        out.append(path)
    return out


@pytest.mark.parametrize("n", [5_000, 100_000])
def test_gcn_delays_and_route_scores(n):
    g = synth_road_graph(n, seed=1)
    m = GcnScorer(seed=2)
    with torch.no_grad():
        ref = m(GcnScorer.adjacency(g), torch.from_numpy(g.features)).numpy()
    hip = GcnScorerHip(m, g, torch.device("cuda:0"))
    got = hip.node_delays().cpu().numpy()
    np.testing.assert_allclose(got, ref, rtol=3e-2, atol=3e-2)
    routes = _random_walks(g, 300)
    ptr, nodes = routes_to_csr(routes)
    sc = hip.score_routes(torch.from_numpy(ptr).cuda(), torch.from_numpy(nodes).cuda()).cpu().numpy()
    np.testing.assert_allclose(sc, score_routes_ref(g, got, routes), rtol=1e-3)


def test_gcn_trained_delays_relative_to_spread():
    """On a TRAINED scorer (outputs spread over the delay range, not sitting at the softplus floor
    like a random init): kernel delays vs the fp32 reference, max error relative to the mean
    absolute deviation of the reference (the K2 criterion), and route-score ranks."""
    from routest_amd.models.gcn_train import train
    from routest_amd.routing.graph import edge_costs
    from routest_amd.serve.eta_service import default_model
    from scipy.stats import spearmanr
    g = synth_road_graph(20_000, seed=8)
    cost = edge_costs(g, default_model(hidden=64, steps=60), device=torch.device("cuda", 0))
    m, _ = train(g, cost, steps=150, lr=5e-3, device="cuda:0")
    with torch.no_grad():
        ref = m(GcnScorer.adjacency(g), torch.from_numpy(g.features)).numpy()
    spread = float(np.abs(ref - ref.mean()).mean())
    assert spread > 0.1, spread                      # a real spread of delay factors
    got = GcnScorerHip(m, g, torch.device("cuda:0")).node_delays().cpu().numpy()
    assert float(np.abs(got - ref).max()) / spread < 0.05
    routes = _random_walks(g, 400, seed=3)
    a, b = score_routes_ref(g, got, routes), score_routes_ref(g, ref, routes)
    assert spearmanr(a, b).correlation > 0.999


def test_gcn_partition_rows_match_full():
    g = synth_road_graph(20_000, seed=3)
    m = GcnScorer(seed=4)
    full = GcnScorerHip(m, g, torch.device("cuda:0")).node_delays().cpu()
    # emulate 4 ranks on one device: each computes its row range; Z gathered by copying slices
    parts = []
    per = (g.num_nodes + 3) // 4
    zs = []
    hs = []
    for r in range(4):
        h = GcnScorerHip(m, g, torch.device("cuda:0"))
        h.rows = (r * per, min(g.num_nodes, (r + 1) * per))
        C = h.C
        r0, r1 = h.rows
        C.gcn_l1_fused(h.X, h.indptr, h.indices, h.values, h.w1, h.b1, h.w2, h.Z, r0, r1)
        zs.append(h.Z[r0:r1].clone())
        hs.append(h)
    Z = torch.cat(zs)
    for h in hs:
        h.Z[:g.num_nodes].copy_(Z)
        r0, r1 = h.rows
        h.C.gcn_spmm_score(h.Z, h.indptr, h.indices, h.values, h.b2, h.wo, h.bo, h.delay, r0, r1)
        parts.append(h.delay[r0:r1].cpu())
    torch.testing.assert_close(torch.cat(parts), full)


@pytest.mark.parametrize("rows", [(0, 30_000), (1_000, 17_777)])
def test_gcn_fused_layer1_bitwise_equals_two_launch_path(rows, monkeypatch):
    """gcn_l1_fused_kernel keeps H1 in LDS; it must reproduce the two-launch path bit for bit."""
    g = synth_road_graph(30_000, seed=5)
    m = GcnScorer(seed=6)
    fused = GcnScorerHip(m, g, torch.device("cuda:0"))
    monkeypatch.setenv("ROUTEST_GCN_FUSED", "0")
    split = GcnScorerHip(m, g, torch.device("cuda:0"))
    assert fused.fused and not split.fused
    r0, r1 = rows
    fused.rows = split.rows = rows
    fused.Z.zero_()
    split.Z.zero_()
    fused.node_delays()
    split.node_delays()
    assert torch.equal(fused.Z[r0:r1], split.Z[r0:r1])
    assert torch.equal(fused.delay[r0:r1], split.delay[r0:r1])


def test_route_score_windows_and_bad_ids():
    """route_score_kernel walks 64-node windows advancing by 63 (the next node's position comes from
    the neighbouring lane): lengths around the window edges, 0/1-node routes, and node ids outside
    [0, N) (their segments add nothing)."""
    g = synth_road_graph(5_000, seed=5)
    m = GcnScorer(seed=6)
    hip = GcnScorerHip(m, g, torch.device("cuda:0"))
    delay = hip.node_delays().cpu().numpy()
    routes = [w[:L] for w, L in zip(_random_walks(g, 9, seed=7, lo=300, hi=301),
                                    [0, 1, 2, 63, 64, 65, 126, 127, 128])]
    bad = list(_random_walks(g, 1, seed=8, lo=100, hi=101)[0])
    bad[10], bad[50] = -1, g.num_nodes + 3
    routes.append(bad)
    ptr, nodes = routes_to_csr(routes)
    got = hip.score_routes(torch.from_numpy(ptr).cuda(), torch.from_numpy(nodes).cuda()).cpu().numpy()
    good = [r for r in routes[:-1]]
    ref = list(score_routes_ref(g, delay, good))
    # the bad route: sum of the segments whose two ends are valid nodes
    segs = [[bad[i], bad[i + 1]] for i in range(len(bad) - 1)
            if 0 <= bad[i] < g.num_nodes and 0 <= bad[i + 1] < g.num_nodes]
    ref.append(sum(score_routes_ref(g, delay, segs)))
    np.testing.assert_allclose(got, np.array(ref, dtype=np.float64), rtol=1e-3, atol=1e-3)
    assert got[0] == 0.0 and got[1] == 0.0
