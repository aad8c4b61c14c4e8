#!/usr/bin/env python3
"""A/B timing of APSP build settings on the C3 workload.

A variant is a set of environment assignments read by the library at each
build (e.g. "SG_APSP_FRONTIER=0"); variants are separated by ';'.  Every
variant must produce the identical table (checked against the first); prints
ms per build and the relaxation-kernel statistics per variant.
    python tools/apsp_variants.py [--nodes 10000] [--variants "SG_APSP_FRONTIER=1;SG_APSP_FRONTIER=0"]
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
    ap.add_argument("--variants", default="SG_APSP_FRONTIER=1;SG_APSP_FRONTIER=0")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--shard-of", type=int, default=1,
                    help="time only rank 0's source-row block of an N-way row sharding (the per-GPU work at N GPUs)")
    a = ap.parse_args()
    import torch

    from shadow_amd import Context, NetworkGraph, synth

    ctx = Context(0, stream=torch.cuda.current_stream().cuda_stream)
    g = synth.ring_chords_graph(a.nodes, a.degree, seed=1)
    net = NetworkGraph(g["n"], g["src"], g["dst"], g["lat"], g["loss"], g["directed"], ctx=ctx)
    n = a.nodes
    used = np.arange(n, dtype=np.uint32)
    r1 = (n + a.shard_of - 1) // a.shard_of  # rank 0's rows
    lat = torch.empty(n * n, dtype=torch.int64, device="cuda")
    loss = torch.empty(n * n, dtype=torch.float32, device="cuda")
    ref = None
    base_env = dict(os.environ)
    variants = a.variants.split(";")

    def set_env(v):
        os.environ.clear()
        os.environ.update(base_env)
        for kv in v.split():
            k, _, val = kv.partition("=")
            os.environ[k] = val

    times = {v: [] for v in variants}
    for _ in range(a.rounds):  # interleaved A/B/A/B...: box-to-box and clock drift hit every variant alike
        for v in variants:
            set_env(v)
            net.build_rows_device(used, 0, r1, lat.data_ptr(), loss.data_ptr(), True)  # warm-up
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.reps):
                net.build_rows_device(used, 0, r1, lat.data_ptr(), loss.data_ptr(), True)
            torch.cuda.synchronize()
            times[v].append((time.perf_counter() - t0) / a.reps * 1e3)
    for v in variants:
        set_env(v)
        ctx.enable_timers(True)
        net.build_rows_device(used, 0, r1, lat.data_ptr(), loss.data_ptr(), True)
        rms, launches, _ = ctx.read_timer("relax")
        oms, _, _ = ctx.read_timer("out")
        ctx.enable_timers(True, count_work=True)
        net.build_rows_device(used, 0, r1, lat.data_ptr(), loss.data_ptr(), True)
        _, _, work = ctx.read_timer("relax")
        ctx.enable_timers(False)
        h = (lat[: 64 * n].cpu().numpy().copy(), loss[: 64 * n].cpu().numpy().copy(),
             lat[(r1 - 64) * n:r1 * n].cpu().numpy().copy())
        same = "ref" if ref is None else all(np.array_equal(x, y) for x, y in zip(h, ref))
        ref = ref or h
        ms = float(np.median(times[v]))
        print(f"variant {v!r}: {ms:8.3f} ms/build (median of {a.rounds}; min {min(times[v]):.3f})  relax {rms:8.3f} ms "
              f"in {launches} launches, out {oms:.3f} ms, {work / 1e9:.3f} G lane-relaxations, {work / max(rms, 1e-9) / 1e6:.1f} G/s  "
              f"identical={same}", flush=True)


if __name__ == "__main__":
    main()
