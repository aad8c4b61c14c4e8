"""Debug: sharded W=2 round, with and without packed rank tables; reports which bucket fails."""
import os, sys
sys.path.insert(0, os.getcwd())
import numpy as np
import torch
sys.path.insert(0, "tests")
import test_dist_gpu as T
from oracle import oracle as O
from shadow_amd import Context
ctx = Context(0)
orig = T.DeviceTable.pack
for mode in sys.argv[1:]:
    T.DeviceTable.pack = orig if mode == "pack" else (lambda self, ctx=None: True)
    try:
        T._run(O, ctx, 2, 30000)
        print(mode, "ok", flush=True)
    except Exception as e:
        print(mode, "FAIL", type(e).__name__, str(e)[:200], flush=True)
