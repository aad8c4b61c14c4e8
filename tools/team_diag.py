#!/usr/bin/env python3
"""Team search (sg_team.hip) diagnostics on the C5-style graph: per setting, the
median build time, the team launches' device time (unbounded / bounded phases),
and the relaxations, messages and supersteps counted in a separate run; every
setting's table compared with the first one's on three 64-row blocks.
python tools/team_diag.py [--nodes 50000] "SG_SSSP_TEAM=4" "SG_SSSP_TEAM=4 SG_SSSP_SEEDS=0" ..."""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=50000)
    ap.add_argument("--degree", type=float, default=8.0)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("settings", nargs="+")
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
    base_env = dict(os.environ)
    ref = None
    for st in a.settings:
        os.environ.clear()
        os.environ.update(base_env)
        for kv in st.split():
            k, _, v = kv.partition("=")
            os.environ[k] = v
        net.build_rows_device(used, 0, n, lat.data_ptr(), loss.data_ptr(), True)
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            net.build_rows_device(used, 0, n, lat.data_ptr(), loss.data_ptr(), True)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        ctx.enable_timers(True)
        net.build_rows_device(used, 0, n, lat.data_ptr(), loss.data_ptr(), True)
        tm = {k: [round(x, 3) if isinstance(x, float) else x for x in ctx.read_timer(k)[:2]]
              for k in ("sssp_team", "sssp_team_bounded", "relax", "plan_sets", "plan_bounds")}
        ctx.enable_timers(True, count_work=True)
        net.build_rows_device(used, 0, n, lat.data_ptr(), loss.data_ptr(), True)
        wk = {k: ctx.read_timer(k)[2] for k in ("sssp_team", "sssp_team_msgs", "sssp_team_steps", "relax")}
        parts = {k[7:]: round(ctx.read_timer(k)[2] / 256, 2) for k in
                 ("team_t_claim", "team_t_setup", "team_t_local", "team_t_remote", "team_t_exchange",
                  "team_t_apply", "team_t_output")}
        ctx.enable_timers(False)
        arcs = len(g["src"]) * (1 if g["directed"] else 2)
        h = [x.cpu().numpy().copy() for x in (lat[:64 * n], loss[(n // 2) * n:(n // 2 + 64) * n], lat[(n - 64) * n:])]
        same = True if ref is None else all(np.array_equal(x, y) for x, y in zip(h, ref))
        ref = ref or h
        print(json.dumps({"setting": st, "ms_median": round(float(np.median(ts)), 2), "timers_ms": tm,
                          "relaxations": wk["sssp_team"], "ms_per_workgroup": parts, "messages": wk["sssp_team_msgs"],
                          "supersteps_per_row": round(wk["sssp_team_steps"] / n, 2),
                          "relax_per_row_per_arc": round(wk["sssp_team"] / (n * arcs), 3),
                          "same_as_first": same}), flush=True)


if __name__ == "__main__":
    main()
