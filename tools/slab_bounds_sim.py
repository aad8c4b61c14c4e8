#!/usr/bin/env python3
"""CPU model: slab passes (Jacobi, frontier = nodes any of the 64 sources changed) with and
without neighbour-row bounds, latency only, on the C5 ring+chords graph.  Prints node passes
per batch.  python tools/slab_bounds_sim.py [n]  """
import numpy as np, sys, time
from scipy.sparse import csr_matrix
from scipy.sparse.csgraph import dijkstra
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from shadow_amd import synth
n = int(sys.argv[1]) if len(sys.argv) > 1 else 50000
g = synth.ring_chords_graph(n, 8.0, seed=1)
s, d, l = g["src"].astype(np.int64), g["dst"].astype(np.int64), (g["lat"] // 1000).astype(np.int64)
keep = s != d
s, d, l = s[keep], d[keep], l[keep]
S = np.concatenate([s, d]); Dd = np.concatenate([d, s]); L = np.concatenate([l, l])
order = np.argsort(Dd, kind="stable"); S, Dd, L = S[order], Dd[order], L[order]
A = csr_matrix((L.astype(float), (S, Dd)), shape=(n, n))
# min over parallel arcs for dijkstra
A.sum_duplicates()
arcs = len(S)
INF = np.int64(1) << 60
def run(srcs, init):
    Dm = init.copy()  # (n, B)
    B = len(srcs)
    Dm[srcs, np.arange(B)] = 0
    front = np.zeros(n, bool); front[srcs] = True
    passes = 0; node_passes = 0; arc_passes = 0
    while front.any():
        passes += 1
        node_passes += front.sum()
        m = front[S]
        arc_passes += m.sum()
        su, dv, w = S[m], Dd[m], L[m]
        cand = Dm[su] + w[:, None]
        # min per destination
        uniq, start = np.unique(dv, return_index=True)
        best = np.minimum.reduceat(cand, start, axis=0)
        old = Dm[uniq]
        newv = np.minimum(old, best)
        ch = (newv < old).any(axis=1)
        Dm[uniq] = newv
        front = np.zeros(n, bool); front[uniq[ch]] = True
    return passes, node_passes, arc_passes
rng = np.random.default_rng(0)
# greedy-ish dominating set: random order, pick nodes not yet dominated
dom = np.zeros(n, bool); covered = np.zeros(n, bool)
nbr_ptr = A.indptr; nbr = A.indices
for v in rng.permutation(n):
    if not covered[v]:
        dom[v] = True; covered[v] = True; covered[nbr[nbr_ptr[v]:nbr_ptr[v+1]]] = True
print("n", n, "arcs", arcs, "dominating", dom.sum(), flush=True)
for trial in range(2):
    b0 = trial * 64 * 97 % n
    srcs = np.array([v for v in range(b0, n) if not dom[v]][:64])
    t = time.time()
    p, npass, ap = run(srcs, np.full((n, 64), INF, np.int64))
    print("unbounded: passes", p, "node-passes/n", round(npass / n, 2), "redundancy", round(ap / arcs, 2), round(time.time()-t,1), flush=True)
    # bounds: for each source, up to 2 dominating neighbours t (arc weight w), D[t] exact
    init = np.full((n, 64), INF, np.int64)
    for i, sv in enumerate(srcs):
        nb = nbr[nbr_ptr[sv]:nbr_ptr[sv+1]]; ww = A.data[nbr_ptr[sv]:nbr_ptr[sv+1]].astype(np.int64)
        sel = np.where(dom[nb])[0][:2]
        if len(sel) == 0: continue
        dt = dijkstra(A, indices=nb[sel]).astype(np.int64)
        ub = (dt + ww[sel][:, None]).min(axis=0)
        init[:, i] = ub + 1
    p, npass, ap = run(srcs, init)
    print("bounded:   passes", p, "node-passes/n", round(npass / n, 2), "redundancy", round(ap / arcs, 2), flush=True)
