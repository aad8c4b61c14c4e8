#!/usr/bin/env python3
"""One warm C3 routing build (for rocprofv3 PMC passes on the search kernel)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from shadow_amd import Context, NetworkGraph, synth

    n = int(os.environ.get("SG_NODES", "10000"))
    ctx = Context(0, stream=torch.cuda.current_stream().cuda_stream)
    g = synth.ring_chords_graph(n, 8.0, seed=1)
    net = NetworkGraph(g["n"], g["src"], g["dst"], g["lat"], g["loss"], g["directed"], ctx=ctx)
    used = np.arange(n, dtype=np.uint32)
    lat = torch.empty(n * n, dtype=torch.int64, device="cuda")
    loss = torch.empty(n * n, dtype=torch.float32, device="cuda")
    for _ in range(2):
        net.build_rows_device(used, 0, n, lat.data_ptr(), loss.data_ptr(), True)
    torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()
