"""The sharded path over real RCCL on the GPU (backend "nccl", world size 1).

tools/rccl_check.py runs in a child process of its own (RCCL wants one process
per rank, and two ranks cannot share a device): the APSP row-block
all_gather_into_tensor and ShardedDelivery.round (sg_deliver_source,
exchange_round's all-gather + all_to_all_single on device tensors,
sg_deliver_bucket), each checked against the single-GPU path inside the child.
The N > 1 exchange logic itself is covered with gloo in tests/test_dist_cpu.py."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_rccl_world1_sharded_round_and_allgather():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", LOCAL_RANK="0",
               WORLD_SIZE="1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tools", "rccl_check.py")], env=env, cwd=ROOT,
                       capture_output=True, text=True, timeout=150)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")][-1]
    res = json.loads(line)
    assert res["ok"] and res["backend"] == "nccl" and res["records"] > 0
    print(line)
