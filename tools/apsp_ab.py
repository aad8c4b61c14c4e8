#!/usr/bin/env python3
"""A/B of APSP build settings on a ring + chords graph (default C5: 50k nodes, mean degree 8):
    python tools/apsp_ab.py --nodes 50000 --variants "SG_APSP_BUCKET=0;SG_BUCKET_SHIFT=22"
Times each variant in interleaved rounds (a rebuild on the same device graph), checks that every
variant's table equals the first one's on the device, and prints the timers of one counting run
(relaxations; the bucketed search's per-row buckets / entries with SG_BUCKET_DIAG=1)."""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=50000)
    ap.add_argument("--degree", type=float, default=8.0)
    ap.add_argument("--rows", type=int, default=0, help="build rows [0, rows) only (0: the whole table)")
    ap.add_argument("--variants", default="")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--no-check", action="store_true", help="timing diagnostics: tables may differ")
    a = ap.parse_args()
    import torch

    from shadow_amd import Context, NetworkGraph, synth

    ctx = Context(0, stream=torch.cuda.current_stream().cuda_stream)
    g = synth.ring_chords_graph(a.nodes, a.degree, seed=1)
    net = NetworkGraph(g["n"], g["src"], g["dst"], g["lat"], g["loss"], g["directed"], ctx=ctx)
    n = a.nodes
    n_arcs = int(np.count_nonzero(g["src"] != g["dst"])) * (1 if g["directed"] else 2)
    rows = a.rows or n
    used = np.arange(n, dtype=np.uint32)
    lat = torch.empty(rows * n, dtype=torch.int64, device="cuda")
    loss = torch.empty(rows * n, dtype=torch.float32, device="cuda")
    ref = None
    base = dict(os.environ)
    variants = a.variants.split(";")
    times = {v: [] for v in variants}

    def set_env(v):
        os.environ.clear()
        os.environ.update(base)
        for kv in v.split():
            k, _, val = kv.partition("=")
            os.environ[k] = val

    for r in range(a.rounds):
        for v in variants:
            set_env(v)
            net.build_rows_device(used, 0, rows, lat.data_ptr(), loss.data_ptr(), True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.reps):
                net.build_rows_device(used, 0, rows, lat.data_ptr(), loss.data_ptr(), True)
            torch.cuda.synchronize()
            times[v].append((time.perf_counter() - t0) / a.reps * 1e3)
            if r == 0:
                if ref is None:
                    ref = (lat.clone(), loss.clone())
                else:
                    same = torch.equal(lat, ref[0]) and torch.equal(loss.view(torch.int32), ref[1].view(torch.int32))
                    print(f"variant {v!r}: table {'identical' if same else 'DIFFERS'}", flush=True)
                    assert same or a.no_check, v
            print(f"round {r} variant {v!r}: {times[v][-1]:9.3f} ms/build", flush=True)
    for v in variants:
        set_env(v + " SG_BUCKET_DIAG=1")
        ctx.enable_timers(True, count_work=True)
        net.build_rows_device(used, 0, rows, lat.data_ptr(), loss.data_ptr(), True)
        torch.cuda.synchronize()
        parts = []
        for k in ("sssp_bucket", "relax", "sssp", "sssp_bounded"):
            ms, launches, work = ctx.read_timer(k)
            if launches:
                parts.append(f"{k} {ms:.3f} ms / {launches} launches, {work / 1e9:.3f} G relaxations "
                             f"({work / (rows * max(1, n_arcs)):.3f} x rows*arcs)")
        ent = ctx.read_timer("sssp_bucket_entries")[2]
        if ent:
            parts.append(f"{ent / (rows * n):.3f} arena entries per cell")
        ctx.enable_timers(False)
        print(f"variant {v!r}: median {np.median(times[v]):9.3f} ms/build; " + "; ".join(parts), flush=True)


if __name__ == "__main__":
    main()
