#!/usr/bin/env python3
"""Where a one-shot row-block build's time goes (C3 graph, default 1,250 rows = one rank of an
8-way split): sg_net_create alone, the build on a fresh graph, a rebuild on the same graph, and
sg_net_destroy, each timed on the host with a device synchronize.  python tools/oneshot_parts.py"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from shadow_amd import Context, NetworkGraph, synth

    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 1250
    ctx = Context(0, stream=torch.cuda.current_stream().cuda_stream)
    g = synth.ring_chords_graph(10000, 8.0, seed=1)
    n = g["n"]
    used = np.arange(n, dtype=np.uint32)
    bl = torch.empty(rows * n, dtype=torch.int64, device="cuda")
    bf = torch.empty(rows * n, dtype=torch.float32, device="cuda")
    parts = {"create": [], "build_fresh": [], "rebuild": [], "destroy": [], "one_shot": []}
    for it in range(12):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        net = NetworkGraph(g["n"], g["src"], g["dst"], g["lat"], g["loss"], g["directed"], ctx=ctx)
        net._ensure_net()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        net.build_rows_device(used, 0, rows, bl.data_ptr(), bf.data_ptr(), True)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        net.build_rows_device(used, 0, rows, bl.data_ptr(), bf.data_ptr(), True)
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        net.close()
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        net2 = NetworkGraph(g["n"], g["src"], g["dst"], g["lat"], g["loss"], g["directed"], ctx=ctx)
        net2.build_rows_device(used, 0, rows, bl.data_ptr(), bf.data_ptr(), True)
        net2.close()
        torch.cuda.synchronize()
        t5 = time.perf_counter()
        if it >= 2:
            for k, v in zip(parts, (t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4)):
                parts[k].append(v * 1e3)
    print({k: round(float(np.median(v)), 4) for k, v in parts.items()}, flush=True)


if __name__ == "__main__":
    main()
