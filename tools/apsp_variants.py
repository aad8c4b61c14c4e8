#!/usr/bin/env python3
"""A/B timing of the APSP kernel variants (SG_APSP_VARIANT) on the C3 workload.

Every variant must produce the identical table (checked against the first);
prints ms per build and the relaxation-kernel statistics per variant.
    python tools/apsp_variants.py [--nodes 10000] [--variants 32xf,64,...]
"""
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
    ap.add_argument("--variants", default="64,64x,64f,64xf,32,32x,32f,32xf")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch

    from shadow_amd import Context, NetworkGraph, synth

    ctx = Context(0, stream=torch.cuda.current_stream().cuda_stream)
    g = synth.ring_chords_graph(a.nodes, a.degree, seed=1)
    net = NetworkGraph(g["n"], g["src"], g["dst"], g["lat"], g["loss"], g["directed"], ctx=ctx)
    n = a.nodes
    used = np.arange(n, dtype=np.uint32)
    lat = torch.empty(n * n, dtype=torch.int64, device="cuda")
    loss = torch.empty(n * n, dtype=torch.float32, device="cuda")
    ref = None
    for v in a.variants.split(","):
        os.environ["SG_APSP_VARIANT"] = v
        net.build_rows_device(used, 0, n, lat.data_ptr(), loss.data_ptr(), True)  # warm-up
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            net.build_rows_device(used, 0, n, lat.data_ptr(), loss.data_ptr(), True)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / a.reps * 1e3
        ctx.enable_timers(True)
        net.build_rows_device(used, 0, n, lat.data_ptr(), loss.data_ptr(), True)
        rms, launches, work = ctx.read_timer("relax_packed")
        ctx.enable_timers(False)
        h = (lat[: 64 * n].cpu().numpy().copy(), loss[: 64 * n].cpu().numpy().copy(),
             lat[-64 * n:].cpu().numpy().copy())
        same = "ref" if ref is None else all(np.array_equal(x, y) for x, y in zip(h, ref))
        ref = ref or h
        print(f"variant {v:5s}: {ms:8.3f} ms/build  relax {rms:8.3f} ms in {launches} launches, "
              f"{work / 1e9:.3f} G lane-relaxations, {work / max(rms, 1e-9) / 1e6:.1f} G/s  identical={same}",
              flush=True)


if __name__ == "__main__":
    main()
