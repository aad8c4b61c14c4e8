#!/usr/bin/env python3
"""Experiment: how the grouping of sources into 64-source batches changes the
relaxation work of the APSP build (C3 workload).

The rows of a batch share one frontier (a node is re-gathered in a pass when any
of the batch's 64 sources improved it), so batches of sources that are close in
the latency metric should converge in fewer active (batch, node) rows.  The
order is passed as the `nodes` list: rows come out permuted, which is fine for
timing.  Prints ms per build and lane-relaxations per ordering.
    python tools/apsp_order.py [--nodes 10000]
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def orders(g, n, which):
    import scipy.sparse as sp
    from scipy.sparse.csgraph import breadth_first_order, depth_first_order, dijkstra, reverse_cuthill_mckee

    w = g["lat"].astype(np.float64) / 1e6
    keep = g["src"] != g["dst"]
    s, d, w = g["src"][keep], g["dst"][keep], w[keep]
    if not g["directed"]:
        s, d, w = np.concatenate([s, d]), np.concatenate([d, s]), np.concatenate([w, w])
    A = sp.csr_matrix((w, (s, d)), shape=(n, n))  # (parallel arcs sum: an approximation, fine for an order)
    out = {}
    if "ident" in which:
        out["ident"] = np.arange(n)
    if "random" in which:
        out["random"] = np.random.default_rng(5).permutation(n)
    if "bfs" in which:
        out["bfs"] = breadth_first_order(A, 0, directed=False, return_predecessors=False)
    if "rcm" in which:
        out["rcm"] = reverse_cuthill_mckee(A, symmetric_mode=True)
    if "sptdfs" in which:  # DFS preorder of the shortest-path tree from node 0
        _, pred = dijkstra(A, directed=False, indices=0, return_predecessors=True)
        T = sp.coo_matrix((np.ones(n - 1), (pred[1:].clip(0), np.arange(1, n))), shape=(n, n)).tocsr()
        out["sptdfs"] = depth_first_order(T, 0, directed=True, return_predecessors=False)
    if "cluster" in which:  # greedy: seed = lowest unassigned index, batch = its 63 nearest unassigned nodes
        t0 = time.perf_counter()
        left = np.ones(n, bool)
        order = []
        while left.any():
            s = int(np.argmax(left))
            lim = 0.05
            while True:
                d = dijkstra(A, directed=False, indices=s, limit=lim)
                cand = np.nonzero(left & np.isfinite(d))[0]
                if len(cand) >= 64 or lim > 100:
                    break
                lim *= 2
            cand = cand[np.argsort(d[cand], kind="stable")][:64]
            order.extend(cand.tolist())
            left[cand] = False
        out["cluster"] = np.array(order)
        print(f"cluster order: {time.perf_counter() - t0:.2f} s on the host", flush=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=10000)
    ap.add_argument("--degree", type=float, default=8.0)
    ap.add_argument("--which", default="ident,random,bfs,rcm,sptdfs,cluster")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch

    from shadow_amd import Context, NetworkGraph, synth

    ctx = Context(0, stream=torch.cuda.current_stream().cuda_stream)
    g = synth.ring_chords_graph(a.nodes, a.degree, seed=1)
    n = a.nodes
    net = NetworkGraph(g["n"], g["src"], g["dst"], g["lat"], g["loss"], g["directed"], ctx=ctx)
    lat = torch.empty(n * n, dtype=torch.int64, device="cuda")
    loss = torch.empty(n * n, dtype=torch.float32, device="cuda")
    for name, o in orders(g, n, a.which.split(",")).items():
        used = np.ascontiguousarray(o, dtype=np.uint32)
        assert len(np.unique(used)) == n
        net.build_rows_device(used, 0, n, lat.data_ptr(), loss.data_ptr(), True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            net.build_rows_device(used, 0, n, lat.data_ptr(), loss.data_ptr(), True)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / a.reps * 1e3
        ctx.enable_timers(True)
        net.build_rows_device(used, 0, n, lat.data_ptr(), loss.data_ptr(), True)
        rms, launches, _ = ctx.read_timer("relax")
        ctx.enable_timers(True, count_work=True)
        net.build_rows_device(used, 0, n, lat.data_ptr(), loss.data_ptr(), True)
        _, _, work = ctx.read_timer("relax")
        ctx.enable_timers(False)
        print(f"order {name:8s}: {ms:8.3f} ms/build  relax {rms:7.3f} ms in {launches} launches, "
              f"{work / 1e9:6.3f} G lane-relaxations", flush=True)


if __name__ == "__main__":
    main()
