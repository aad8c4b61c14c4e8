#!/usr/bin/env python3
"""Per-row statistics of the LDS-resident search (SG_SSSP_DIAG) on the C3 graph for
several bucket widths (whole table or a row block): cycles in the search and in the row write-out, phases, far
scans, relaxations per row.  python tools/sssp_diag.py [--nodes 10000] [--deltas 25e6,1e9]"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=10000)
    ap.add_argument("--degree", type=float, default=8.0)
    ap.add_argument("--deltas", default="25e6,50e6,4e9")
    ap.add_argument("--rows", default="", help="r0:r1, a rank's row block (default: every row)")
    a = ap.parse_args()
    import torch

    from shadow_amd import Context, NetworkGraph, synth

    ctx = Context(0, stream=torch.cuda.current_stream().cuda_stream)
    g = synth.ring_chords_graph(a.nodes, a.degree, seed=1)
    net = NetworkGraph(g["n"], g["src"], g["dst"], g["lat"], g["loss"], g["directed"], ctx=ctx)
    n = a.nodes
    used = np.arange(n, dtype=np.uint32)
    r0, r1 = (int(x) for x in a.rows.split(":")) if a.rows else (0, n)
    lat = torch.empty((r1 - r0) * n, dtype=torch.int64, device="cuda")
    loss = torch.empty((r1 - r0) * n, dtype=torch.float32, device="cuda")
    os.environ["SG_SSSP_DIAG"] = "1"
    for d in a.deltas.split(","):
        os.environ["SG_APSP_DELTA"] = str(int(float(d)))
        net.build_rows_device(used, r0, r1, lat.data_ptr(), loss.data_ptr(), True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        net.build_rows_device(used, r0, r1, lat.data_ptr(), loss.data_ptr(), True)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3
        ctx.enable_timers(True, count_work=True)
        net.build_rows_device(used, r0, r1, lat.data_ptr(), loss.data_ptr(), True)
        ctx.enable_timers(False)
        print(f"delta {d}: {ms:.3f} ms/build", flush=True)


if __name__ == "__main__":
    main()
