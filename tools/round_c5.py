#!/usr/bin/env python3
"""One delivery round at C5 size (100k hosts, 10M packets) on a synthetic 50k x 50k
path table, without the routing build: for kernel profiles of the round alone
(rocprofv3 --pmc passes over it take seconds, not minutes).  The table is random
(latency U[1, 300] ms, loss 0 or U(0, 0.02)); results are not checked here -- the
parity tests and bench.py --config c5 do that.
python tools/round_c5.py [--rounds 5] [--nodes 50000] [--hosts 100000] [--packets 10000000]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--nodes", type=int, default=50000)
    ap.add_argument("--hosts", type=int, default=100000)
    ap.add_argument("--packets", type=int, default=10_000_000)
    a = ap.parse_args()
    import torch

    from shadow_amd import Context, synth
    from shadow_amd.worker import DeviceTable, Deliveries, HostTable, PacketBatch, deliver_round

    ctx = Context(0, stream=torch.cuda.current_stream().cuda_stream)
    n = a.nodes
    g = torch.Generator(device="cuda").manual_seed(1)
    lat = torch.randint(1_000_000, 300_000_000, (n * n,), device="cuda", dtype=torch.int64, generator=g)
    loss = torch.rand(n * n, device="cuda", generator=g) * 0.02
    loss[torch.rand(n * n, device="cuda", generator=g) < 0.8] = 0.0
    table = DeviceTable(lat, loss, n, 0)
    assert table.pack(ctx)
    del lat, loss
    T0 = 946684800 * 10**9
    hosts = synth.make_hosts(a.hosts, n, general_seed=1, exact_seeds=False)
    pk = synth.make_packets(a.packets, hosts, T0 + 10**9, T0 + 10**9 + 10**6, seed=100)
    ht = HostTable(hosts["ip"], hosts["route"], hosts["seed"], ctx=ctx)
    batch = PacketBatch.from_numpy(pk["src"], pk["dst_ip"], pk["payload"], pk["send_time"])
    out = Deliveries.allocate(a.packets, a.hosts)
    for r in range(a.rounds):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        deliver_round(ht, table, batch, T0 + 10**9 + 10**6, 2**63, 0, out=out, ctx=ctx)
        torch.cuda.synchronize()
        print(f"round {r}: {(time.perf_counter() - t0) * 1e3:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
