"""First (cold) and later routing builds of the C3 graph on fresh NetworkGraphs: the cold build
also builds the phase plan (SG_PLAN_DIAG=1 prints its steps).  python tools/cold_build.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from shadow_amd import Context, NetworkGraph, synth
ctx = Context(0, stream=torch.cuda.current_stream().cuda_stream)
g = synth.ring_chords_graph(10000, 8.0, seed=1)
n = 10000
used = np.arange(n, dtype=np.uint32)
lat = torch.empty(n * n, dtype=torch.int64, device="cuda"); loss = torch.empty(n * n, dtype=torch.float32, device="cuda")
for rep in range(3):
    t0 = time.perf_counter()
    net = NetworkGraph(g["n"], g["src"], g["dst"], g["lat"], g["loss"], g["directed"], ctx=ctx)
    torch.cuda.synchronize(); t1 = time.perf_counter()
    for k in range(3):
        ta = time.perf_counter()
        net.build_rows_device(used, 0, n, lat.data_ptr(), loss.data_ptr(), True)
        torch.cuda.synchronize()
        print(f"net {rep} (upload {1e3*(t1-t0):.2f} ms) build {k}: {1e3*(time.perf_counter()-ta):.3f} ms", flush=True)
