#!/usr/bin/env python3
"""A/B of the LDS-resident search's launch knobs on one graph: median build time
per setting, and every setting's table compared bit for bit with the first one's.
python tools/sssp_ab.py [--nodes 10000] [--degree 8] "SG_SSSP_SLOTS=1" "SG_SSSP_SLOTS=2" ..."""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=10000)
    ap.add_argument("--degree", type=float, default=8.0)
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--rows", default="", help="r0:r1, a rank's row block (default: every row)")
    ap.add_argument("settings", nargs="+", help="space-free env assignments, comma separated per setting")
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
    first = None
    for st in a.settings:
        env = dict(kv.split("=", 1) for kv in st.split(",") if kv)
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        net.build_rows_device(used, r0, r1, lat.data_ptr(), loss.data_ptr(), True)
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            net.build_rows_device(used, r0, r1, lat.data_ptr(), loss.data_ptr(), True)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        ctx.enable_timers(True)
        net.build_rows_device(used, r0, r1, lat.data_ptr(), loss.data_ptr(), True)
        tm = {k: round(ctx.read_timer(k)[0], 4) for k in ("sssp", "sssp_bounded", "relax", "relax_wide", "plan_sets", "plan_bounds")}
        ctx.enable_timers(False)
        h = (lat.view(torch.int64).sum().item(), loss.view(torch.int32).to(torch.int64).sum().item())
        if first is None:
            first = (lat.clone(), loss.clone())
            same = True
        else:
            same = bool(torch.equal(first[0], lat) and torch.equal(first[1].view(torch.int32), loss.view(torch.int32)))
        print(json.dumps({"setting": st, "n": n, "ms_median": round(float(np.median(ts)), 4),
                          "ms_min": round(min(ts), 4), "timers_ms": tm, "same_as_first": same, "checksum": h}), flush=True)
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


if __name__ == "__main__":
    main()
