"""bench.py keeps the driver's contract: one JSON line with the required keys,
a roofline object and a CPU baseline, on a small workload (a child process)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_json_contract():
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "1", "--nodes", "1000",
           "--hosts", "5000", "--packets", "50000", "--no-gml", "--no-c2"]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=110)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [x for x in out.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["warmup"] == 1 and d["value"] > 0
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in d["roofline"], k
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in d["cpu_baseline"], k
    assert d["config"]["workload"] and "model" not in d["config"]
    dl = d["delivery"]
    assert dl["value"] > 0 and dl["roofline"]["bound"] == "hbm" and dl["cpu_baseline"]["cores"] >= 1
    assert d["inbound"]["parity_vs_cpu"] is True
