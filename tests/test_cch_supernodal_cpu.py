"""The supernodal customization's algebra on the CPU (numpy emulation of csrc/cch.hip sup_*): basic
customization as blocked tropical elimination of dense fronts and perfect customization as blocked
back substitution give the per-node reference results BIT for bit — packed (weight, middle) words
for basic, f32 weights for perfect — on a small synthetic graph's CCH (csrc/runtime/cch.h topology).

The GPU kernels follow the same block schedule (panel left-looking through the block below, the
block below's trailing update past the current block; product through the part above the block
above, the solve adding that block, then the block's K x K targets top-down), and
tests/test_cch_gpu.py checks the kernels themselves against the per-level kernels and the CPU
reference.  Here the point is the candidate sets: every candidate is one f32 add of two FINAL
operands, so any order of the (exact) minima gives the same bits."""
import numpy as np
import pytest

INF = np.float32(np.inf)
PINF = np.uint64(0x7F800000FFFFFFFF)


def packw(w, p):
    return (np.asarray(w, np.float32).view(np.uint32).astype(np.uint64) << np.uint64(32)) | np.uint64(p)


def wof(x):
    return (np.asarray(x, np.uint64) >> np.uint64(32)).astype(np.uint32).view(np.float32)


@pytest.fixture(scope="module")
def cch():
    from routest_amd.data.graph import synth_road_graph
    import routest_amd._rt as rt
    g = synth_road_graph(1200, seed=3)
    c = rt.CCH(g.indptr, g.indices, g.lat, g.lon, 2)
    a = {k: np.asarray(v) for k, v in c.arrays().items()}
    rng = np.random.default_rng(7)
    cost = rng.uniform(1.0, 60.0, len(g.indices)).astype(np.float32)
    cost[::7] = np.round(cost[::7])            # ties between middles
    return a, cost


def initial(a, cost):
    M = len(a["up_head"])
    up = np.full(M, PINF, np.uint64)
    dn = np.full(M, PINF, np.uint64)
    for e, (arc, d) in enumerate(zip(a["edge_arc"], a["edge_dir"])):
        if arc < 0:
            continue
        w = packw(cost[e], 0x80000000 | e)
        if d:
            dn[arc] = min(dn[arc], w)
        else:
            up[arc] = min(up[arc], w)
    return up, dn


def arc_index(a):
    up_ptr, up_head = a["up_ptr"], a["up_head"]
    return {(x, int(up_head[q])): q for x in range(len(up_ptr) - 1) for q in range(up_ptr[x], up_ptr[x + 1])}


def basic_reference(a, up, dn):
    """Per node in rank order (every lower triangle of an arc has a lower rank): the per-level kernels."""
    up, dn = up.copy(), dn.copy()
    up_ptr, up_head = a["up_ptr"], a["up_head"]
    idx = arc_index(a)
    for z in range(len(up_ptr) - 1):
        arcs = list(range(up_ptr[z], up_ptr[z + 1]))
        for ii, ai in enumerate(arcs):
            for aj in arcs[ii + 1:]:
                t = idx[(int(up_head[ai]), int(up_head[aj]))]
                wu = wof(dn[ai]) + wof(up[aj])
                wd = wof(dn[aj]) + wof(up[ai])
                if wu < INF:
                    up[t] = min(up[t], packw(wu, z))
                if wd < INF:
                    dn[t] = min(dn[t], packw(wd, z))
    return up, dn


def perfect_reference(a, up, dn):
    """Per node top-down (ranks descending): the pull kernels."""
    up_ptr, up_head = a["up_ptr"], a["up_head"]
    idx = arc_index(a)
    pu, pd = wof(up).copy(), wof(dn).copy()
    for x in range(len(up_ptr) - 2, -1, -1):
        arcs = list(range(up_ptr[x], up_ptr[x + 1]))
        for aa in arcs:
            y = int(up_head[aa])
            bu, bd = pu[aa], pd[aa]
            for ac in arcs:
                if ac == aa:
                    continue
                z = int(up_head[ac])
                azy = idx[(min(z, y), max(z, y))]
                zy = pu[azy] if z < y else pd[azy]
                yz = pd[azy] if z < y else pu[azy]
                bu = min(bu, wof(up[ac]) + zy)
                bd = min(bd, yz + wof(dn[ac]))
            pu[aa], pd[aa] = bu, bd
    return pu, pd


def fronts(a, s0):
    """Chains (each node the only child of the next) of >= s0 nodes and their ancestors, levelled."""
    par = a["parent"]
    N = len(par)
    nch = np.bincount(par[par >= 0], minlength=N)
    start = [i for i in range(N) if not (i > 0 and par[i - 1] == i and nch[i] == 1)]
    sid = np.zeros(N, int)
    for s, c0 in enumerate(start):
        end = start[s + 1] if s + 1 < len(start) else N
        sid[c0:end] = s
    size = np.bincount(sid)
    top = [c0 + size[s] - 1 for s, c0 in enumerate(start)]
    spar = [sid[par[t]] if par[t] >= 0 else -1 for t in top]
    dense = np.zeros(len(start), bool)
    for s in range(len(start)):
        q = s
        while size[s] >= s0 and q >= 0 and not dense[q]:
            dense[q] = True
            q = spar[q]
    lev = np.zeros(len(start), int)
    for s in range(len(start)):
        if dense[s] and spar[s] >= 0:
            lev[spar[s]] = max(lev[spar[s]], lev[s] + 1)
    out = []
    for s in np.nonzero(dense)[0]:
        c0, m = start[s], size[s]
        t = top[s]
        U = [int(h) for h in a["up_head"][a["up_ptr"][t]:a["up_ptr"][t + 1]]]
        out.append((int(lev[s]), c0, int(m), list(range(c0, c0 + m)) + U))
    return out, np.isin(sid, np.nonzero(dense)[0])


def basic_supernodal(a, up, dn, s0, B):
    up, dn = up.copy(), dn.copy()
    idx = arc_index(a)
    F, in_front = fronts(a, s0)
    up_ptr, up_head = a["up_ptr"], a["up_head"]
    # nodes outside the fronts first (rank order), then the fronts level by level
    for z in range(len(up_ptr) - 1):
        if in_front[z]:
            continue
        arcs = list(range(up_ptr[z], up_ptr[z + 1]))
        for ii, ai in enumerate(arcs):
            for aj in arcs[ii + 1:]:
                t = idx[(int(up_head[ai]), int(up_head[aj]))]
                wu = wof(dn[ai]) + wof(up[aj])
                wd = wof(dn[aj]) + wof(up[ai])
                if wu < INF:
                    up[t] = min(up[t], packw(wu, z))
                if wd < INF:
                    dn[t] = min(dn[t], packw(wd, z))
    for level in range(max(f[0] for f in F) + 1):
        for _, c0, m, nodes in [f for f in F if f[0] == level]:
            n = len(nodes)
            arc = np.full((n, n), -1, np.int64)
            D = np.full((n, n), PINF, np.uint64)
            for i in range(n):
                for j in range(n):
                    if i != j and (nodes[min(i, j)], nodes[max(i, j)]) in idx:
                        arc[i, j] = idx[(nodes[min(i, j)], nodes[max(i, j)])]
                        if i < m or j < m:
                            D[i, j] = up[arc[i, j]] if i < j else dn[arc[i, j]]

            def cand(y, p, z):
                w = wof(D[y, p]) + wof(D[p, z])
                return packw(w, c0 + p) if w < INF else PINF
            nb = -(-m // B)
            for b in range(nb):
                k0, k1 = b * B, min(b * B + B, m)
                # panel: left-looking through the block below (its trailing skipped K's rows / columns)
                if b > 0:
                    for y in range(k0, n):
                        for z in range(k0, n):
                            if y != z and (y < k1 or z < k1):
                                for p in range(k0 - B, k0):
                                    D[y, z] = min(D[y, z], cand(y, p, z))
                for p in range(k0, k1):
                    for y in range(p + 1, n):
                        for z in range(p + 1, n):
                            if y != z and (y < k1 or z < k1):
                                D[y, z] = min(D[y, z], cand(y, p, z))
                # trailing: past the block above K (every target for the last block)
                zr0 = min(k1 + B, m) if b + 1 < nb else k1
                for y in range(zr0, n):
                    for z in range(zr0, n):
                        if y != z:
                            for p in range(k0, k1):
                                D[y, z] = min(D[y, z], cand(y, p, z))
            for i in range(n):
                for j in range(i + 1, n):
                    t = arc[i, j]
                    if t < 0:
                        continue
                    if i < m:
                        up[t], dn[t] = D[i, j], D[j, i]
                    else:                                   # U x U: the atomicMin into the arc
                        up[t] = min(up[t], D[i, j])
                        dn[t] = min(dn[t], D[j, i])
    return up, dn


def perfect_supernodal(a, up, dn, s0, B):
    idx = arc_index(a)
    F, in_front = fronts(a, s0)
    pu, pd = wof(up).copy(), wof(dn).copy()
    for level in range(max(f[0] for f in F), -1, -1):
        for _, c0, m, nodes in [f for f in F if f[0] == level]:
            n = len(nodes)
            arc = np.full((n, n), -1, np.int64)
            Db = np.full((n, n), INF, np.float32)
            P = np.full((n, n), INF, np.float32)
            for i in range(n):
                for j in range(n):
                    if i != j and (nodes[min(i, j)], nodes[max(i, j)]) in idx:
                        t = idx[(nodes[min(i, j)], nodes[max(i, j)])]
                        arc[i, j] = t
                        if i < m or j < m:
                            Db[i, j] = wof(up[t]) if i < j else wof(dn[t])
                            P[i, j] = Db[i, j]
                        else:
                            P[i, j] = pu[t] if i < j else pd[t]
            nb = -(-m // B)
            for b in range(nb - 1, -1, -1):
                k0, k1 = b * B, min(b * B + B, m)
                zlo = min(k1 + B, m) if b + 1 < nb else k1
                # product through the part above the block above K (no data from that block's K x K)
                for x in range(k0, k1):
                    for y in range(k1, n):
                        for z in range(zlo, n):
                            P[x, y] = min(P[x, y], Db[x, z] + P[z, y])
                            P[y, x] = min(P[y, x], P[y, z] + Db[z, x])
                # the solve: the block above K first, then top-down through K
                for x in range(k0, k1):
                    for y in range(k1, n):
                        for z in range(k1, zlo):
                            P[x, y] = min(P[x, y], Db[x, z] + P[z, y])
                            P[y, x] = min(P[y, x], P[y, z] + Db[z, x])
                for z in range(k1 - 1, k0, -1):
                    for x in range(k0, z):
                        for y in range(k1, n):
                            P[x, y] = min(P[x, y], Db[x, z] + P[z, y])
                            P[y, x] = min(P[y, x], P[y, z] + Db[z, x])
                # K x K: the part above K, then top-down through K
                for x in range(k0, k1):
                    for y in range(x + 1, k1):
                        for z in range(k1, n):
                            P[x, y] = min(P[x, y], Db[x, z] + P[z, y])
                            P[y, x] = min(P[y, x], P[y, z] + Db[z, x])
                for x in range(k1 - 2, k0 - 1, -1):
                    for y in range(x + 1, k1):
                        for z in range(x + 1, k1):
                            if z != y:
                                P[x, y] = min(P[x, y], Db[x, z] + P[z, y])
                                P[y, x] = min(P[y, x], P[y, z] + Db[z, x])
            for i in range(m):
                for j in range(i + 1, n):
                    t = arc[i, j]
                    if t >= 0:
                        pu[t], pd[t] = P[i, j], P[j, i]
    # the other nodes top-down (their ancestors inside fronts are final)
    up_ptr, up_head = a["up_ptr"], a["up_head"]
    for x in range(len(up_ptr) - 2, -1, -1):
        if in_front[x]:
            continue
        arcs = list(range(up_ptr[x], up_ptr[x + 1]))
        for aa in arcs:
            y = int(up_head[aa])
            bu, bd = pu[aa], pd[aa]
            for ac in arcs:
                if ac == aa:
                    continue
                z = int(up_head[ac])
                azy = idx[(min(z, y), max(z, y))]
                zy = pu[azy] if z < y else pd[azy]
                yz = pd[azy] if z < y else pu[azy]
                bu = min(bu, wof(up[ac]) + zy)
                bd = min(bd, yz + wof(dn[ac]))
            pu[aa], pd[aa] = bu, bd
    return pu, pd


@pytest.mark.parametrize("s0,B", [(3, 4), (8, 8)])
def test_supernodal_blocked_algebra_is_bit_identical(cch, s0, B):
    a, cost = cch
    F, in_front = fronts(a, s0)
    assert len(F) >= 2 and max(f[2] for f in F) > B          # several fronts, several blocks
    up0, dn0 = initial(a, cost)
    ru, rd = basic_reference(a, up0, dn0)
    su, sd = basic_supernodal(a, up0, dn0, s0, B)
    assert np.array_equal(ru, su) and np.array_equal(rd, sd)
    pu, pd = perfect_reference(a, ru, rd)
    qu, qd = perfect_supernodal(a, ru, rd, s0, B)
    assert np.array_equal(pu.view(np.uint32), qu.view(np.uint32))
    assert np.array_equal(pd.view(np.uint32), qd.view(np.uint32))
