#!/usr/bin/env python3
"""One-shot C3 builds (fresh sg_net + plan + search + destroy), timed on the host, for a
kernel/copy trace: run under rocprofv3 --kernel-trace --memory-copy-trace and read the gaps
with --analyze DIR.  python tools/build_timeline.py [--nodes 10000] [--reps 5]"""
import argparse
import csv
import glob
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def analyze(d):
    ks = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][-40:]))
    for f in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "COPY " + r.get("Direction", "")))
    ks.sort()
    # builds: split at the first k_net_count of each build
    starts = [i for i, k in enumerate(ks) if "k_net_count" in k[2]]
    for bi, s in enumerate(starts[-2:]):
        e = starts[starts.index(s) + 1] if starts.index(s) + 1 < len(starts) else len(ks)
        t0 = ks[s][0]
        print(f"build {bi}: {(ks[e - 1][1] - t0) / 1e3:.1f} us from the first kernel to the last end")
        prev_end = t0
        for k in ks[s:e]:
            print(f"  +{(k[0] - t0) / 1e3:8.1f} gap {(k[0] - prev_end) / 1e3:7.1f}  dur {(k[1] - k[0]) / 1e3:8.1f}  {k[2]}")
            prev_end = max(prev_end, k[1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=10000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--analyze", default="")
    a = ap.parse_args()
    if a.analyze:
        analyze(a.analyze)
        return
    import torch

    from shadow_amd import Context, NetworkGraph, synth

    ctx = Context(0, stream=torch.cuda.current_stream().cuda_stream)
    g = synth.ring_chords_graph(a.nodes, 8.0, seed=1)
    n = a.nodes
    used = np.arange(n, dtype=np.uint32)
    lat = torch.empty(n * n, dtype=torch.int64, device="cuda")
    loss = torch.empty(n * n, dtype=torch.float32, device="cuda")
    ts, parts = [], []
    for _ in range(a.reps + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        net = NetworkGraph(g["n"], g["src"], g["dst"], g["lat"], g["loss"], g["directed"], ctx=ctx)
        t1 = time.perf_counter()
        net._ensure_net()  # sg_net_create: validation, staging copy, upload launches (returns unsynchronised)
        t2 = time.perf_counter()
        net.build_rows_device(used, 0, n, lat.data_ptr(), loss.data_ptr(), True)
        t3 = time.perf_counter()
        net.close()
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        ts.append((t4 - t0) * 1e3)
        parts.append([round((b - a_) * 1e6, 1) for a_, b in ((t0, t1), (t1, t2), (t2, t3), (t3, t4))])
    print("one-shot build ms:", [round(t, 3) for t in ts], flush=True)
    print("host us [NetworkGraph(), sg_net_create, build call, close+sync]:", parts[1:], flush=True)


if __name__ == "__main__":
    main()
