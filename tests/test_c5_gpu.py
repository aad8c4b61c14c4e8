"""C5 at full size (BASELINE configs[4]): the 50k-node ring + chords graph,
every node used, its whole 2.5·10^9-cell routing table, and a 10M-packet round over 100k
hosts -- unsharded, and sharded by destination over 8 ranks emulated on one GPU.

* The table: every cell is checked by the oracle's fixed-point certificate
  (oracle/sg_oracle.c sgo_check_fixed_point: the equations petgraph's Dijkstra's result is
  the unique solution of, graph/mod.rs:183-228), and one 64-row batch out of every 16 against
  the oracle's Dijkstra itself.  So the round oracle below is fed a table proven to be the
  reference's, not merely the GPU's.
* The round is compared with the oracle's send_packet restatement (worker.rs:322-397,
  event.rs:84-155) on every output: status, arrival time, event id, per-destination order and
  offsets, the round minima, and every host's RNG stream and event counter.  Gather indices run
  past 2^31 cells here.
* The sharded round (north_star: delivery sharded by destination host, configs[4]): 8 rank
  blocks of 6,250 rows, each built by its own sg_net and sg_routing_build call as a rank would
  (worker.rs:597-607 hand-off, manager.rs:482-487 global minimum), hosts partitioned by
  HostPartition, each rank's source phase on its block, the exchange by concatenation (what the
  all-to-all moves), in the exact and the padded (fixed-split) protocol, and bucketing at the
  destination owner -- equal to the one oracle round above.
"""
import os

import numpy as np
import pytest

from shadow_amd import NetworkGraph, synth
from shadow_amd.dist import (HostPartition, RECORD_DTYPE, gpu_bucket_phase, gpu_bucket_phase_padded,
                             gpu_source_phase, gpu_source_phase_padded, next_cap, row_range)
from shadow_amd.worker import DeviceTable, HostTable, PacketBatch, deliver_round

pytestmark = pytest.mark.gpu
N = 50_000
W = 8  # ranks of configs[4]
T0 = 946684800 * 10**9  # EmulatedTime SIMULATION_START
THREADS = min(16, os.cpu_count() or 1)


@pytest.fixture(scope="module")
def c5(ctx):
    import torch

    g = synth.ring_chords_graph(N, 8.0, seed=1)
    net = NetworkGraph(g["n"], g["src"], g["dst"], g["lat"], g["loss"], g["directed"], ctx=ctx)
    used = np.arange(N, dtype=np.uint32)
    lat = torch.empty(N * N, dtype=torch.int64, device="cuda")
    loss = torch.empty(N * N, dtype=torch.float32, device="cuda")
    net.build_rows_device(used, 0, N, lat.data_ptr(), loss.data_ptr(), True)
    torch.cuda.synchronize()
    yield g, used, lat, loss
    del lat, loss
    torch.cuda.empty_cache()


@pytest.fixture(scope="module")
def c5_host(c5):
    """The whole table in host memory (30 GB), for the certificate and the round oracle."""
    g, used, lat, loss = c5
    lat_h = lat.cpu().numpy().view(np.uint64).reshape(N, N)
    loss_h = loss.cpu().numpy().reshape(N, N)
    yield lat_h, loss_h
    del lat_h, loss_h


def test_c5_table_every_cell_fixed_point(c5, c5_host, oracle):
    """All 2.5·10^9 cells: the table solves compute_shortest_paths' fixed-point equations (which
    have one solution, the reference's), and its diagonal is each node's self-loop."""
    g, used, _, _ = c5
    lat_h, loss_h = c5_host
    bad, first = oracle.check_fixed_point(N, g["src"], g["dst"], g["lat"], g["loss"], False, used, lat_h, loss_h,
                                          threads=THREADS)
    assert bad == 0, f"{bad} cells off the fixed point, first at (row, col) = {first}"


def test_c5_table_every_16th_batch(c5, oracle):
    """One 64-row batch out of every 16 of the whole 50k-row table (49 batches), every cell
    bit-exact against the oracle's Dijkstra."""
    g, used, lat, loss = c5
    batches = range(0, (N + 63) // 64, 16)
    assert len(batches) == 49
    for b in batches:
        r0, r1 = 64 * b, min(N, 64 * b + 64)
        rc, olat, oloss, _ = oracle.shortest_paths(g["n"], g["src"], g["dst"], g["lat"], g["loss"], False, used,
                                                   rows=(r0, r1), threads=THREADS)
        assert rc == 0
        glat = lat[r0 * N:r1 * N].cpu().numpy().view(np.uint64).reshape(r1 - r0, N)
        gloss = loss[r0 * N:r1 * N].cpu().numpy().view(np.uint32).reshape(r1 - r0, N)
        assert np.array_equal(glat, olat), f"latency mismatch in rows [{r0}, {r1})"
        assert np.array_equal(gloss, oloss.view(np.uint32)), f"loss mismatch in rows [{r0}, {r1})"


PACKET_SEED = 5


@pytest.fixture(scope="module")
def c5_round(c5, c5_host, oracle, ctx):
    """The 10M-packet round's inputs and the oracle's result for them, from the certified
    table (one oracle run for every round test of the module)."""
    g, used, lat, loss = c5
    lat_h, loss_h = c5_host
    hosts = synth.make_hosts(100_000, N, general_seed=1, exact_seeds=True)
    start, end = T0 + 10**9, T0 + 10**9 + 10**6
    pk = synth.make_packets(10_000_000, hosts, start, end, seed=PACKET_SEED, p_unknown_dst=0.001)
    ht = HostTable(hosts["ip"], hosts["route"], hosts["seed"], ctx=ctx)
    rng0, ctr0 = ht.get_state()
    del ht
    orng, octr = rng0.copy(), ctr0.copy()
    want = oracle.deliver_round(end, 2**63, 0, pk["src"], pk["dst_ip"], pk["payload"], pk["send_time"], hosts["ip"],
                                hosts["route"], lat_h, loss_h, orng, octr, threads=THREADS)
    yield hosts, pk, end, (rng0, ctr0), (want, orng, octr)


@pytest.mark.parametrize("packed", [True, False])
def test_c5_round_on_full_table(c5, c5_round, ctx, packed):
    """10M packets from 100k hosts (node h mod 50k) delivered from the full 50k table,
    in both table forms (packed 8-byte path keys and the two arrays)."""
    g, used, lat, loss = c5
    hosts, pk, end, (rng0, ctr0), (want, rng, ctr) = c5_round
    table = DeviceTable(lat, loss, N)
    if packed:
        assert table.pack(ctx)
    ht = HostTable(hosts["ip"], hosts["route"], hosts["seed"], ctx=ctx)
    hr, hc = ht.get_state()
    assert np.array_equal(hr, rng0) and np.array_equal(hc, ctr0)  # the oracle ran from this state
    out = deliver_round(ht, table, PacketBatch.from_numpy(pk["src"], pk["dst_ip"], pk["payload"], pk["send_time"]),
                        end, 2**63, 0, ctx=ctx)
    got = out.to_numpy(len(pk["src"]))
    grng, gctr = ht.get_state()
    del out, table
    assert want["delivered"] > 9_000_000
    for k in ("status", "deliver_time", "event_id", "dst_offsets", "dst_order"):
        assert np.array_equal(got[k], want[k]), k
    assert got["delivered"] == want["delivered"]
    assert got["min_deliver"] == want["min_deliver"] and got["min_lat"] == want["min_lat"]
    assert np.array_equal(grng, rng) and np.array_equal(gctr, ctr)


# ---------------------------------------------------------------------------------------------
# configs[4]: the same round sharded by destination host over 8 ranks (emulated on one GPU)
# ---------------------------------------------------------------------------------------------
@pytest.fixture(scope="module")
def c5_blocks(c5, ctx, oracle):
    """Rank r's 6,250-row block, built as rank r builds it: its own sg_net (sg_net_create) and
    one sg_routing_build over rows [r0, r1) -- checked bit for bit against the certified whole
    table, and its first and last 32 rows against the oracle's Dijkstra."""
    import torch

    g, used, lat, loss = c5
    blocks = []
    for r in range(W):
        r0, r1, per = row_range(N, W, r)
        net = NetworkGraph(g["n"], g["src"], g["dst"], g["lat"], g["loss"], g["directed"], ctx=ctx)
        bl = torch.empty((r1 - r0) * N, dtype=torch.int64, device="cuda")
        bf = torch.empty((r1 - r0) * N, dtype=torch.float32, device="cuda")
        net.build_rows_device(used, r0, r1, bl.data_ptr(), bf.data_ptr(), True)
        torch.cuda.synchronize()
        net.close()
        assert torch.equal(bl, lat[r0 * N:r1 * N]), f"rank {r}: latency block differs from the whole table"
        assert torch.equal(bf.view(torch.int32), loss[r0 * N:r1 * N].view(torch.int32)), f"rank {r}: loss block"
        for a, b in ((r0, r0 + 32), (r1 - 32, r1)):
            rc, olat, oloss, _ = oracle.shortest_paths(g["n"], g["src"], g["dst"], g["lat"], g["loss"], False, used,
                                                       rows=(a, b), threads=THREADS)
            assert rc == 0
            assert np.array_equal(bl[(a - r0) * N:(b - r0) * N].cpu().numpy().view(np.uint64).reshape(b - a, N), olat)
            assert np.array_equal(bf[(a - r0) * N:(b - r0) * N].cpu().numpy().view(np.uint32).reshape(b - a, N),
                                  oloss.view(np.uint32))
        blocks.append((r0, r1, bl, bf))
    yield blocks
    del blocks
    torch.cuda.empty_cache()


def _expected_for_rank(want, hosts_of_d):
    """The oracle's per-destination lists of rank d's hosts, in slot order, and their offsets."""
    off = want["dst_offsets"].astype(np.int64)
    cnt = off[hosts_of_d + 1] - off[hosts_of_d]
    starts = np.repeat(off[hosts_of_d], cnt)
    within = np.arange(cnt.sum()) - np.repeat(np.cumsum(cnt) - cnt, cnt)
    return want["dst_order"][starts + within].astype(np.int64), np.concatenate([[0], np.cumsum(cnt)])


@pytest.mark.parametrize("mode", ["exact", "padded"])
def test_c5_sharded_round_8_ranks(c5_blocks, c5_round, ctx, mode):
    """configs[4] at its size: 8 ranks, each with its row block (odd ranks from packed path
    keys), its hosts' 1.25M packets through the source phase, the records exchanged by
    concatenation -- exact (counts first) or padded (one fixed-split block per rank pair, cap
    from the previous round's largest pair count) -- and bucketed on the owner: statuses, times,
    event ids, every destination's order and offsets, the global minima, and every host's RNG
    stream and counter equal the one unsharded oracle round."""
    import torch

    hosts, pk, end, (rng0, ctr0), (want, rng, ctr) = c5_round
    part = HostPartition(hosts["route"], N, W)
    owner_of_pkt = part.owner[pk["src"]]
    sels = [np.nonzero(owner_of_pkt == r)[0] for r in range(W)]
    assert sum(len(s) for s in sels) == len(pk["src"])
    assert min(part.n_local(r) for r in range(W)) == 100_000 // W  # route = node h mod 50k: even shares
    owner_dev = torch.from_numpy(part.owner.view(np.int32)).cuda()
    local_dev = torch.from_numpy(part.local.view(np.int32)).cuda()
    # cap of a padded round: from the largest pair count of a round before (here: this round's
    # counts, computed on the host, plus next_cap's slack -- what ShardedDelivery carries over)
    pair = np.zeros((W, W), np.int64)
    dst_host = np.full(len(pk["src"]), -1, np.int64)
    by_ip = np.argsort(hosts["ip"])
    dl = want["status"] == 0  # SG_PKT_DELIVERED
    dst_host[dl] = by_ip[np.searchsorted(hosts["ip"][by_ip], pk["dst_ip"][dl])]
    assert np.array_equal(hosts["ip"][dst_host[dl]], pk["dst_ip"][dl])
    np.add.at(pair, (owner_of_pkt[dl], part.owner[dst_host[dl]]), 1)
    cap = next_cap(int(pair.max()))
    srcs, stats = [], []
    for r in range(W):
        r0, r1, bl, bf = c5_blocks[r]
        table = DeviceTable(bl, bf, N, r0)
        if r % 2:
            assert table.pack(ctx)
        ht = HostTable(hosts["ip"], hosts["route"], hosts["seed"], ctx=ctx)
        sel = sels[r]
        batch = PacketBatch.from_numpy(pk["src"][sel], pk["dst_ip"][sel], pk["payload"][sel], pk["send_time"][sel])
        if mode == "exact":
            s = gpu_source_phase(ctx, ht, table, batch, end, 2**63, 0, owner_dev, W)
            assert s.send_counts == [int(x) for x in pair[r]]
            stats.append((s.n_delivered, s.min_deliver_time_ns, s.min_used_latency_ns))
            keep = dict(send=s.send[:sum(s.send_counts)].clone(), counts=list(s.send_counts))
        else:
            s = gpu_source_phase_padded(ctx, ht, table, batch, end, 2**63, 0, owner_dev, W, cap)
            keep = dict(send_padded=s.send_padded.clone(), xrow=s.xrow.clone())
        n = len(sel)
        st = s.status[:n].cpu().numpy()
        dt = s.deliver_time_ns[:n].cpu().numpy().view(np.uint64)
        ev = s.event_id[:n].cpu().numpy().view(np.uint64)
        assert np.array_equal(st, want["status"][sel]), f"rank {r}: status"
        assert np.array_equal(dt, want["deliver_time"][sel]), f"rank {r}: deliver time"
        assert np.array_equal(ev, want["event_id"][sel]), f"rank {r}: event id"
        grng, gctr = ht.get_state()
        mine = part.hosts_of[r]
        assert np.array_equal(grng[mine], rng[mine]) and np.array_equal(gctr[mine], ctr[mine]), f"rank {r}: streams"
        # the other ranks' hosts were not touched by this rank's source phase
        others = np.setdiff1d(np.arange(hosts["n"]), mine)
        assert np.array_equal(grng[others], rng0[others]) and np.array_equal(gctr[others], ctr0[others])
        del ht, table, s
        srcs.append(keep)
    if mode == "exact":
        g = (sum(x[0] for x in stats), min(x[1] for x in stats), min(x[2] for x in stats))
        assert g == (want["delivered"], want["min_deliver"], want["min_lat"])
        xall = None
    else:
        xall = torch.cat([k["xrow"] for k in srcs])
        xa = xall.cpu().numpy().view(np.uint64).reshape(W, 3 + W)
        assert np.array_equal(xa[:, 3:].astype(np.int64), pair)
        assert int(xa[:, 3:].max()) <= cap  # no overflow: one exchange
    for d in range(W):
        if mode == "exact":
            parts, origin = [], []
            for sidx, k in enumerate(srcs):
                o = int(sum(k["counts"][:d]))
                parts.append(k["send"][o:o + k["counts"][d]])
                origin.append(np.full(k["counts"][d], sidx, np.int64))
            recv = torch.cat(parts).contiguous()
            origin = np.concatenate(origin)
            order, offsets = gpu_bucket_phase(ctx, recv, recv.shape[0], local_dev, hosts["n"], part.n_local(d))
        else:
            recv = torch.cat([k["send_padded"][d * cap:(d + 1) * cap] for k in srcs]).contiguous()
            origin = np.repeat(np.arange(W), cap)
            order, offsets, gst, rcnt, pmax = gpu_bucket_phase_padded(ctx, recv, cap, xall, d, local_dev, hosts["n"],
                                                                      part.n_local(d))
            assert gst == (want["delivered"], want["min_deliver"], want["min_lat"])
            assert rcnt == [int(x) for x in pair[:, d]] and pmax == int(pair.max())
        rec = recv.cpu().numpy().view(RECORD_DTYPE).ravel()
        ordr = order.cpu().numpy().view(np.uint32).astype(np.int64)
        offs = offsets.cpu().numpy().view(np.uint32).astype(np.int64)
        exp, exp_off = _expected_for_rank(want, part.hosts_of[d].astype(np.int64))
        assert np.array_equal(offs[:len(exp_off)], exp_off), f"rank {d}: destination offsets"
        assert len(ordr) == len(exp)
        picked = rec[ordr]
        org = origin[ordr]
        glob = np.empty(len(ordr), np.int64)
        for sidx in range(W):
            m = org == sidx
            glob[m] = sels[sidx][picked["packet"][m]]
        assert np.array_equal(glob, exp), f"rank {d}: per-destination order"
        assert np.array_equal(picked["deliver_time_ns"], want["deliver_time"][glob])
        assert np.array_equal(picked["event_id"], want["event_id"][glob])
        assert np.array_equal(picked["dst_host"].astype(np.int64), dst_host[glob])
