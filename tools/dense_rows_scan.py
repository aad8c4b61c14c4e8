"""The dense search's launch time against the rows it computes (C2 graph): tells a latency-bound
launch (flat in rows while they fit the chip at once) from a throughput-bound one.
usage: python tools/dense_rows_scan.py [ROWS ...]   (env knobs of sg_dense.hip apply)"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from shadow_amd import Context, NetworkGraph, synth

    rows_list = [int(x) for x in sys.argv[1:]] or [64, 128, 256, 512, 768, 1024, 1200]
    ctx = Context()
    g = synth.complete_graph(1200, seed=1)
    net = NetworkGraph(g["n"], g["src"], g["dst"], g["lat"], g["loss"], False, ctx=ctx)
    n = g["n"]
    used = np.arange(n, dtype=np.uint32)
    lat = torch.empty(n * n, dtype=torch.int64, device="cuda")
    loss = torch.empty(n * n, dtype=torch.float32, device="cuda")
    net.build_rows_device(used, 0, n, lat.data_ptr(), loss.data_ptr(), True)
    for r in rows_list:
        for _ in range(3):
            net.build_rows_device(used, 0, r, lat.data_ptr(), loss.data_ptr(), True)
        ctx.enable_timers(True)
        for _ in range(20):
            net.build_rows_device(used, 0, r, lat.data_ptr(), loss.data_ptr(), True)
        ms, k, _ = ctx.read_timer("sssp_dense")
        ctx.enable_timers(False)
        print(f"rows {r:5d}  launch {ms / max(k, 1) * 1e3:8.1f} us  ({k} launches)", flush=True)


if __name__ == "__main__":
    main()
