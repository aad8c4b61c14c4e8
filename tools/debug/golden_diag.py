"""Diagnose golden-vector mismatches of the routing build under env variants."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from shadow_amd import Context, NetworkGraph  # noqa: E402

z = np.load("tests/golden/routing_small.npz")
ctx = Context(0)
for env in ["SG_APSP_OUT_TPB=1", "SG_APSP_OUT_TPB=2", "SG_APSP_OUT_TPB=1 SG_APSP_PASS_CHUNK=1"]:
    for k in ("SG_APSP_OUT_TPB", "SG_APSP_PASS_CHUNK"):
        os.environ.pop(k, None)
    for kv in env.split():
        k, v = kv.split("=")
        os.environ[k] = v
    for name in sorted({k.split(".")[0] for k in z.files}):
        net = NetworkGraph(int(z[f"{name}.n"][0]), z[f"{name}.src"], z[f"{name}.dst"], z[f"{name}.lat"],
                           z[f"{name}.loss"], bool(z[f"{name}.directed"][0]), ctx=ctx)
        used = z[f"{name}.used"]
        t = net.compute_shortest_paths(used)
        bad = np.nonzero((t.latency_ns != z[f"{name}.out_lat"]) |
                         (t.packet_loss.view(np.uint32) != z[f"{name}.out_loss"].view(np.uint32)))
        nb = len(bad[0])
        msg = "" if not nb else f" first {bad[0][:5]} {bad[1][:5]} got {t.latency_ns[bad][:3]} want {z[f'{name}.out_lat'][bad][:3]}"
        print(f"{env:40s} {name:16s} n={net.n_nodes} used={len(used)} mismatches={nb}{msg}", flush=True)
