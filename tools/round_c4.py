#!/usr/bin/env python3
"""C4 delivery round timing (1M packets, 100k hosts, random 10k x 10k table) under
several environment settings, for A/B of the bucketing knobs; no parity check here
(tests and bench.py do that).  python tools/round_c4.py "SG_SB_TARGET=1024" ..."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from shadow_amd import Context, synth
    from shadow_amd.worker import DeviceTable, Deliveries, HostTable, PacketBatch, deliver_round

    ctx = Context(0, stream=torch.cuda.current_stream().cuda_stream)
    n, H, P = 10000, 100000, 1_000_000
    g = torch.Generator(device="cuda").manual_seed(1)
    lat = torch.randint(1_000_000, 300_000_000, (n * n,), device="cuda", dtype=torch.int64, generator=g)
    loss = torch.rand(n * n, device="cuda", generator=g) * 0.02
    table = DeviceTable(lat, loss, n, 0)
    assert table.pack(ctx)
    T0 = 946684800 * 10**9
    hosts = synth.make_hosts(H, n, general_seed=1, exact_seeds=False)
    pk = synth.make_packets(P, hosts, T0 + 10**9, T0 + 10**9 + 10**6, seed=100)
    ht = HostTable(hosts["ip"], hosts["route"], hosts["seed"], ctx=ctx)
    batch = PacketBatch.from_numpy(pk["src"], pk["dst_ip"], pk["payload"], pk["send_time"])
    out = Deliveries.allocate(P, H)
    for st in sys.argv[1:] or [""]:
        env = dict(kv.split("=", 1) for kv in st.split(",") if kv)
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        for _ in range(5):
            deliver_round(ht, table, batch, T0 + 10**9 + 10**6, 2**63, 0, out=out, ctx=ctx)
        torch.cuda.synchronize()
        ts = []
        for _ in range(20):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            deliver_round(ht, table, batch, T0 + 10**9 + 10**6, 2**63, 0, out=out, ctx=ctx)
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        ctx.enable_timers(True)
        deliver_round(ht, table, batch, T0 + 10**9 + 10**6, 2**63, 0, out=out, ctx=ctx)
        km = {k: round(ctx.read_timer(k)[0], 4) for k in ("seg_bounds", "walk", "scatter", "scatter2", "sort_small")}
        ctx.enable_timers(False)
        print(f"{st or 'default'}: round {sorted(ts)[len(ts) // 2]:.4f} ms, kernels {km}", flush=True)
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


if __name__ == "__main__":
    main()
