"""Regenerate the golden fixtures in tests/golden/ (run from the repo root).

Sources of truth, in order:
  * reference_kat.json -- values copied from the reference's own tests and
    config (graph/mod.rs:519-533, 564-651; configuration.rs:1366-1380) and the
    upstream rand_xoshiro xoshiro256++ vector [external]; hand-written here.
  * routing_small.npz / deliver_small.npz / rng_vectors.json -- produced by the
    CPU oracle (oracle/sg_oracle.c), itself pinned against reference_kat.json
    and scipy (tests/test_oracle.py).  They freeze the oracle's output so that
    GPU parity is also checked against committed vectors.

    python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402
from shadow_amd import synth  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))


def routing_cases():
    cases = {}
    cases["dir16_parallel"] = synth.ring_chords_graph(16, 4.0, seed=3, directed=True, parallel=0.3)
    cases["und64"] = synth.ring_chords_graph(64, 6.0, seed=4)
    cases["und200_lossy"] = synth.ring_chords_graph(200, 8.0, seed=5)
    cases["complete48"] = synth.complete_graph(48, seed=6)
    # latencies near/above 2^34 ns exercise the wide (u64) kernel
    big = synth.ring_chords_graph(40, 4.0, seed=7, lat_lo_us=3_000_000, lat_hi_us=9_000_000)
    cases["und40_bigLat"] = big
    out = {}
    for name, g in cases.items():
        used = np.arange(g["n"], dtype=np.uint32)
        if name == "und200_lossy":  # a used subset in scrambled order (HashSet order is arbitrary)
            used = np.random.default_rng(1).permutation(g["n"])[:150].astype(np.uint32)
        rc, lat, loss, _ = O.shortest_paths(g["n"], g["src"], g["dst"], g["lat"], g["loss"], g["directed"], used,
                                            threads=8)
        assert rc == 0, (name, rc)
        for k in ("src", "dst", "lat", "loss"):
            out[f"{name}.{k}"] = g[k]
        out[f"{name}.n"] = np.array([g["n"]], np.uint32)
        out[f"{name}.directed"] = np.array([int(g["directed"])], np.uint8)
        out[f"{name}.used"] = used
        out[f"{name}.out_lat"] = lat
        out[f"{name}.out_loss"] = loss
    np.savez_compressed(os.path.join(HERE, "routing_small.npz"), **out)


def deliver_case():
    g = synth.ring_chords_graph(50, 6.0, seed=11)
    used = np.arange(50, dtype=np.uint32)
    rc, lat, loss, _ = O.shortest_paths(50, g["src"], g["dst"], g["lat"], g["loss"], False, used)
    assert rc == 0
    # make some paths very lossy so drops happen
    loss = loss.copy()
    loss[::3, ::2] = np.float32(0.5)
    hosts = synth.make_hosts(300, 50, general_seed=1)
    start, end = 946684800 * 10**9 + 10**9, 946684800 * 10**9 + 10**9 + 10**6
    pk = synth.make_packets(10000, hosts, start, end, seed=12, p_unknown_dst=0.02, hot_dst=7, p_hot=0.05)
    pk["send_time"][-5:] = end + 10**9  # past sim end
    rng = np.stack([O.xoshiro_seed(int(s)) for s in hosts["seed"]]).astype(np.uint64)
    ctr = np.zeros(300, np.uint64)
    rng0, ctr0 = rng.copy(), ctr.copy()
    res = O.deliver_round(end, end + 10**9, start + 500_000, pk["src"], pk["dst_ip"], pk["payload"], pk["send_time"],
                          hosts["ip"], hosts["route"], lat, loss, rng, ctr)
    np.savez_compressed(os.path.join(HERE, "deliver_small.npz"), tab_lat=lat, tab_loss=loss, host_ip=hosts["ip"],
                        host_route=hosts["route"], host_seed=hosts["seed"], rng0=rng0, ctr0=ctr0,
                        src=pk["src"], dst_ip=pk["dst_ip"], payload=pk["payload"], send_time=pk["send_time"],
                        round=np.array([end, end + 10**9, start + 500_000], np.uint64), rng1=rng, ctr1=ctr,
                        status=res["status"], deliver_time=res["deliver_time"], event_id=res["event_id"],
                        dst_order=res["dst_order"], dst_offsets=res["dst_offsets"],
                        stats=np.array([res["delivered"], res["min_deliver"], res["min_lat"]], np.uint64))


def rng_vectors():
    v = {}
    for seed in (0, 1, 42, 2**63 + 5):
        s = O.xoshiro_seed(seed)
        v[str(seed)] = {"state": [int(x) for x in s],
                        "f64": [O.xoshiro_next_f64(s) for _ in range(8)]}
    v["host_seed_general1"] = {f"host{h:06d}": O.host_seed(1, f"host{h:06d}") for h in range(4)}
    with open(os.path.join(HERE, "rng_vectors.json"), "w") as f:
        json.dump(v, f, indent=1)


if __name__ == "__main__":
    routing_cases()
    deliver_case()
    rng_vectors()
    print("golden fixtures written to", HERE)
