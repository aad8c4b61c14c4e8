#!/usr/bin/env python3
"""The multi-GPU code path over real RCCL on one GPU (world size 1, backend "nccl").

Every check runs twice: with the collectives through the library's C ABI
(shadow_amd.comm.Comm: sg_comm_allgather_rows, sg_comm_exchange_padded,
sg_comm_alltoallv_records, sg_comm_allgather_u64 -- RCCL on the context's stream,
the calls the Rust caller of INTEGRATION.md makes) and through torch.distributed.

Run as a child process by tests/test_rccl_gpu.py (RCCL needs a process of its
own per rank; two ranks cannot share a device).  It drives, on device tensors:
  * the APSP row-block all-gather (all_gather_into_tensor, as bench.py does),
  * ShardedDelivery.round: sg_deliver_source, exchange_round (the all-gather of
    counts and round scalars, then all_to_all_single of the records) and
    sg_deliver_bucket,
and checks them against the single-GPU path (sg_routing_build, deliver_round).
Prints one JSON line: ok, and the exchange's timings.

Sizes: the defaults are a 600-node graph, 4,000 hosts and 200k packets (the -m gpu test);
--c5 runs BASELINE configs[4]'s sizes through the same calls: the 50k-node table (2.5·10^9
cells, compared on the device with a second build instead of a host copy), 100k hosts and
10M packets.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
T0 = 946684800 * 10**9


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--c5", action="store_true", help="configs[4] sizes: 50k nodes, 100k hosts, 10M packets")
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    size = dict(nodes=50_000, degree=8.0, hosts=100_000, packets=10_000_000) if a.c5 else \
        dict(nodes=600, degree=6.0, hosts=4000, packets=200_000)
    import torch
    import torch.distributed as dist

    from shadow_amd import Context, NetworkGraph, synth
    from shadow_amd.comm import Comm
    from shadow_amd.dist import RECORD_DTYPE, HostPartition, ShardedDelivery, exchange_round
    from shadow_amd.worker import DeviceTable, HostTable, PacketBatch, deliver_round

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
    ctx = Context(0, stream=torch.cuda.current_stream().cuda_stream)
    comm = Comm.from_torch(ctx, dist)
    assert comm.n_ranks == 1 and comm.rank == 0
    res = {}
    for name, exch in (("sg_comm", comm), ("torch", dist)):
        res[name] = check(ctx, exch, dist, torch, size, a.reps)
    comm.close()
    print(json.dumps({"ok": True, "backend": dist.get_backend(), "size": size, **res["sg_comm"],
                      "torch_collectives": res["torch"]}), flush=True)
    dist.destroy_process_group()


def check(ctx, exch, dist, torch, size, reps):
    from shadow_amd import NetworkGraph, synth
    from shadow_amd.comm import is_comm
    from shadow_amd.dist import RECORD_DTYPE, HostPartition, ShardedDelivery, exchange_round
    from shadow_amd.worker import DeviceTable, HostTable, PacketBatch, deliver_round

    # ---- APSP rows + the RCCL all-gather of the row blocks
    n = size["nodes"]
    g = synth.ring_chords_graph(n, size["degree"], seed=9)
    net = NetworkGraph(g["n"], g["src"], g["dst"], g["lat"], g["loss"], g["directed"], ctx=ctx)
    used = np.arange(n, dtype=np.uint32)
    mine_lat = torch.empty(n * n, dtype=torch.int64, device="cuda")
    mine_loss = torch.empty(n * n, dtype=torch.float32, device="cuda")
    net.build_rows_device(used, 0, n, mine_lat.data_ptr(), mine_loss.data_ptr(), True)
    if is_comm(exch):  # in place: the rank's block is its slice of the table
        full_lat, full_loss = mine_lat, mine_loss
        exch.allgather_rows(full_lat, full_loss, n, n)
    else:
        full_lat = torch.empty_like(mine_lat)
        full_loss = torch.empty_like(mine_loss)
        dist.all_gather_into_tensor(full_lat, mine_lat)
        dist.all_gather_into_tensor(full_loss, mine_loss)
    torch.cuda.synchronize()
    if n <= 4096:
        ref = net.compute_shortest_paths(used)
        assert np.array_equal(full_lat.cpu().numpy().view(np.uint64).reshape(n, n), ref.latency_ns)
        assert np.array_equal(full_loss.cpu().numpy().view(np.uint32).reshape(n, n), ref.packet_loss.view(np.uint32))
    else:  # (configs[4]: a second build, compared on the device; its parity: tests/test_c5_gpu.py)
        ref_lat, ref_loss = torch.empty_like(mine_lat), torch.empty_like(mine_loss)
        net.build_rows_device(used, 0, n, ref_lat.data_ptr(), ref_loss.data_ptr(), True)
        torch.cuda.synchronize()
        assert torch.equal(full_lat, ref_lat) and torch.equal(full_loss.view(torch.int32), ref_loss.view(torch.int32))
        del ref_lat, ref_loss
        if full_lat is not mine_lat:
            del mine_lat, mine_loss

    # ---- a sharded delivery round through RCCL vs the single-GPU round
    hosts = synth.make_hosts(size["hosts"], n, general_seed=9, exact_seeds=size["hosts"] <= 10_000)
    start, end = T0 + 10**9, T0 + 10**9 + 10**6
    pk = synth.make_packets(size["packets"], hosts, start, end, seed=9, p_unknown_dst=0.01)
    table = DeviceTable(full_lat, full_loss, n, 0)
    batch = PacketBatch.from_numpy(pk["src"], pk["dst_ip"], pk["payload"], pk["send_time"])
    part = HostPartition(hosts["route"], n, 1)
    ht_s = HostTable(hosts["ip"], hosts["route"], hosts["seed"], ctx=ctx)
    sd = ShardedDelivery(ctx, ht_s, table, part, 0, 1, dist=exch)
    src, recv, recv_counts, order, offsets = sd.round(batch, end, 2**63, start + 100_000)
    ht = HostTable(hosts["ip"], hosts["route"], hosts["seed"], ctx=ctx)
    out = deliver_round(ht, table, batch, end, 2**63, start + 100_000)
    want = out.to_numpy(len(pk["src"]))
    P = len(pk["src"])
    assert np.array_equal(src.status[:P].cpu().numpy(), want["status"])
    assert np.array_equal(src.deliver_time_ns[:P].cpu().numpy().view(np.uint64), want["deliver_time"])
    assert np.array_equal(src.event_id[:P].cpu().numpy().view(np.uint64), want["event_id"])
    rec = recv.cpu().numpy().view(RECORD_DTYPE).ravel()
    glob = rec["packet"].astype(np.int64)[order.cpu().numpy().view(np.uint32)]
    assert np.array_equal(glob, want["dst_order"].astype(np.int64))
    assert np.array_equal(offsets.cpu().numpy().view(np.uint32), want["dst_offsets"])
    assert sd.last_stats == (want["delivered"], want["min_deliver"], want["min_lat"])
    g1, g2 = ht_s.get_state(), ht.get_state()
    assert np.array_equal(g1[0], g2[0]) and np.array_equal(g1[1], g2[1])

    # ---- the fixed-split exchange (padded=True): round 1 exact (sizes the blocks), then padded
    ht_p = HostTable(hosts["ip"], hosts["route"], hosts["seed"], ctx=ctx)
    sdp = ShardedDelivery(ctx, ht_p, table, part, 0, 1, dist=exch, padded=True)
    ht_r = HostTable(hosts["ip"], hosts["route"], hosts["seed"], ctx=ctx)
    for k in range(3):
        src_p, recv_p, rc_p, order_p, offs_p = sdp.round(batch, end, 2**63, start + 100_000)
        ref = deliver_round(ht_r, table, batch, end, 2**63, start + 100_000).to_numpy(P)
        assert sdp.last_mode == ("exact" if k == 0 else "padded"), sdp.last_mode
        assert np.array_equal(src_p.status[:P].cpu().numpy(), ref["status"])
        rec_p = recv_p.cpu().numpy().view(RECORD_DTYPE).ravel()
        glob_p = rec_p["packet"].astype(np.int64)[order_p.cpu().numpy().view(np.uint32)]
        assert np.array_equal(glob_p, ref["dst_order"].astype(np.int64)), k
        assert np.array_equal(offs_p.cpu().numpy().view(np.uint32), ref["dst_offsets"])
        assert sdp.last_stats == (ref["delivered"], ref["min_deliver"], ref["min_lat"])
    g1, g2 = ht_p.get_state(), ht_r.get_state()
    assert np.array_equal(g1[0], g2[0]) and np.array_equal(g1[1], g2[1])

    # ---- timings: the whole sharded round, and exchange_round alone (its one host sync)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        sd.round(batch, end, 2**63, start + 100_000)
    torch.cuda.synchronize()
    t_round = (time.perf_counter() - t0) / reps
    stats = (int(src.n_delivered), int(src.min_deliver_time_ns), int(src.min_used_latency_ns))
    t0 = time.perf_counter()
    for _ in range(reps):
        exchange_round(src.send, src.send_counts, stats, 0, exch)
    torch.cuda.synchronize()
    t_ex = (time.perf_counter() - t0) / reps
    t0 = time.perf_counter()
    for _ in range(reps):
        deliver_round(ht, table, batch, end, 2**63, start + 100_000, out=out)
    torch.cuda.synchronize()
    t_single = (time.perf_counter() - t0) / reps
    t0 = time.perf_counter()
    for _ in range(reps):
        sdp.round(batch, end, 2**63, start + 100_000)
    torch.cuda.synchronize()
    t_padded = (time.perf_counter() - t0) / reps
    assert sdp.last_mode == "padded"
    # the sharded round's phases one at a time (each call returns synchronised)
    from shadow_amd.dist import gpu_bucket_phase, gpu_source_phase
    ph = {"source": 0.0, "exchange": 0.0, "bucket": 0.0}
    for _ in range(reps):
        t0 = time.perf_counter()
        s = gpu_source_phase(ctx, ht_s, table, batch, end, 2**63, start + 100_000, sd.owner_dev, 1)
        t1 = time.perf_counter()
        rv, rc, _ = exchange_round(s.send, s.send_counts, (int(s.n_delivered), int(s.min_deliver_time_ns),
                                                           int(s.min_used_latency_ns)), 0, exch)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        gpu_bucket_phase(ctx, rv, int(sum(rc)), sd.local_dev, len(part.local), part.n_local(0))
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        ph["source"] += (t1 - t0) / reps
        ph["exchange"] += (t2 - t1) / reps
        ph["bucket"] += (t3 - t2) / reps
    return {"packets": P, "records": int(sum(recv_counts)),
            "sharded_round_ms": round(t_round * 1e3, 4), "exchange_round_ms": round(t_ex * 1e3, 4),
            "sharded_round_padded_ms": round(t_padded * 1e3, 4), "padded_cap": sdp.cap,
            "single_gpu_round_ms": round(t_single * 1e3, 4),
            "phases_ms": {k: round(v * 1e3, 4) for k, v in ph.items()}}


if __name__ == "__main__":
    main()
