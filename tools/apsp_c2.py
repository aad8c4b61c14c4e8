#!/usr/bin/env python3
"""A/B of APSP build settings on the C2 workload (1,200-node complete graph):
    python tools/apsp_c2.py --variants "SG_APSP_B=64;SG_APSP_NPW=2 SG_APSP_STAGE=64 SG_APSP_GROUP=4"
Prints ms per build per variant (interleaved rounds) and checks identical tables."""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=1200)
    ap.add_argument("--variants", default="SG_APSP_B=64")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    import torch

    from shadow_amd import Context, NetworkGraph, synth

    ctx = Context(0, stream=torch.cuda.current_stream().cuda_stream)
    g = synth.complete_graph(a.nodes, seed=1)
    net = NetworkGraph(g["n"], g["src"], g["dst"], g["lat"], g["loss"], g["directed"], ctx=ctx)
    n = a.nodes
    used = np.arange(n, dtype=np.uint32)
    lat = torch.empty(n * n, dtype=torch.int64, device="cuda")
    loss = torch.empty(n * n, dtype=torch.float32, device="cuda")
    base = dict(os.environ)
    variants = a.variants.split(";")
    times = {v: [] for v in variants}
    ref = None

    def set_env(v):
        os.environ.clear()
        os.environ.update(base)
        for kv in v.split():
            k, _, val = kv.partition("=")
            os.environ[k] = val

    for _ in range(a.rounds):
        for v in variants:
            set_env(v)
            net.build_rows_device(used, 0, n, lat.data_ptr(), loss.data_ptr(), True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.reps):
                net.build_rows_device(used, 0, n, lat.data_ptr(), loss.data_ptr(), True)
            torch.cuda.synchronize()
            times[v].append((time.perf_counter() - t0) / a.reps * 1e3)
            h = (lat.cpu().numpy().copy(), loss.cpu().numpy().copy())
            same = ref is None or all(np.array_equal(x, y) for x, y in zip(h, ref))
            ref = ref or h
            assert same, v
    for v in variants:
        set_env(v)
        ctx.enable_timers(True)
        net.build_rows_device(used, 0, n, lat.data_ptr(), loss.data_ptr(), True)
        rms, launches, _ = ctx.read_timer("relax")
        ctx.enable_timers(False)
        print(f"variant {v!r}: {np.median(times[v]):8.3f} ms/build  relax {rms:7.3f} ms in {launches} launches",
              flush=True)


if __name__ == "__main__":
    main()
