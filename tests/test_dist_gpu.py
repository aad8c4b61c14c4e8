"""GPU parity of the sharded delivery kernels (sg_deliver_source / sg_deliver_bucket).

W ranks are emulated in one process on one GPU: each rank holds its routing
row shard and runs the source phase for the hosts it owns; the exchange is a
concatenation (the all-to-all itself is covered by tests/test_dist_cpu.py with
gloo).  The result must equal one oracle round over all packets.
"""
import numpy as np
import pytest

from shadow_amd import synth
from shadow_amd.dist import HostPartition, RECORD_DTYPE, ShardedDelivery, row_range
from shadow_amd.worker import DeviceTable, HostTable, PacketBatch

pytestmark = pytest.mark.gpu
T0 = 946684800 * 10**9


def _world(oracle, n_nodes=90, n_hosts=1500, seed=3):
    g = synth.ring_chords_graph(n_nodes, 6.0, seed=seed)
    used = np.arange(n_nodes, dtype=np.uint32)
    rc, lat, loss, _ = oracle.shortest_paths(n_nodes, g["src"], g["dst"], g["lat"], g["loss"], False, used, threads=8)
    assert rc == 0
    loss = loss.copy()
    loss[1::2, ::3] = np.float32(0.4)
    hosts = synth.make_hosts(n_hosts, n_nodes, general_seed=seed)
    return lat, loss, hosts


def _run(oracle, ctx, W, n_packets, hot=None, seed=1, p_hot=0.1, skip=False):
    import torch

    lat, loss, hosts = _world(oracle, seed=seed)
    nu = lat.shape[0]
    part = HostPartition(hosts["route"], nu, W)
    start, end = T0 + 10**9, T0 + 10**9 + 10**6
    pk = synth.make_packets(n_packets, hosts, start, end, seed=seed + 10, p_unknown_dst=0.01,
                            hot_dst=-1 if hot is None else hot, p_hot=0.0 if hot is None else p_hot)
    rs = np.random.default_rng(seed).integers(0, 4, n_packets).astype(np.uint32) if skip else None
    owner_of_pkt = part.owner[pk["src"]]
    ranks = []
    for r in range(W):
        r0, r1, per = row_range(nu, W, r)
        sel = np.nonzero(owner_of_pkt == r)[0]
        ht = HostTable(hosts["ip"], hosts["route"], hosts["seed"], ctx=ctx)
        dl = torch.from_numpy(np.ascontiguousarray(lat[r0:r1]).view(np.int64).ravel()).cuda()
        df = torch.from_numpy(np.ascontiguousarray(loss[r0:r1]).ravel()).cuda()
        table = DeviceTable(dl, df, nu, r0)
        if r % 2:  # odd ranks gather from the packed path-key table (row block offset r0)
            assert table.pack(ctx)
        batch = PacketBatch.from_numpy(pk["src"][sel], pk["dst_ip"][sel], pk["payload"][sel], pk["send_time"][sel],
                                       rng_skip=None if rs is None else rs[sel])
        ranks.append(dict(sel=sel, ht=ht, table=table, batch=batch))
    # source phases
    sends = []
    for r, R in enumerate(ranks):
        sd = ShardedDelivery(ctx, R["ht"], R["table"], part, r, W)
        src = sd.source_fn(ctx, R["ht"], R["table"], R["batch"], end, 2**63, start + 200_000, sd.owner_dev, W)
        R["src"], R["sd"] = src, sd
        sends.append(src)
    # exchange by concatenation: rank d receives segment d of every sender, in sender order
    results = []
    for d, R in enumerate(ranks):
        parts, origin = [], []
        for s, src in enumerate(sends):
            off = int(sum(src.send_counts[:d]))
            cnt = src.send_counts[d]
            parts.append(src.send[off:off + cnt])
            origin += [s] * cnt
        recv = torch.cat(parts) if parts else torch.empty((0, 4), dtype=torch.int64, device="cuda")
        order, offsets = R["sd"].bucket_fn(ctx, recv.contiguous(), recv.shape[0], R["sd"].local_dev,
                                           len(part.local), part.n_local(d))
        results.append((recv, np.array(origin, np.int64), order, offsets))
    # oracle over all packets
    ht0 = HostTable(hosts["ip"], hosts["route"], hosts["seed"], ctx=ctx)
    rng, ctr = ht0.get_state()
    want = oracle.deliver_round(end, 2**63, start + 200_000, pk["src"], pk["dst_ip"], pk["payload"], pk["send_time"],
                                hosts["ip"], hosts["route"], lat, loss, rng, ctr, rng_skip=rs)
    # per-packet outputs + host streams
    for r, R in enumerate(ranks):
        sel = R["sel"]
        assert np.array_equal(R["src"].status[:len(sel)].cpu().numpy(), want["status"][sel])
        assert np.array_equal(R["src"].deliver_time_ns[:len(sel)].cpu().numpy().view(np.uint64), want["deliver_time"][sel])
        assert np.array_equal(R["src"].event_id[:len(sel)].cpu().numpy().view(np.uint64), want["event_id"][sel])
        grng, gctr = R["ht"].get_state()
        mine = part.hosts_of[r]
        assert np.array_equal(grng[mine], rng[mine]) and np.array_equal(gctr[mine], ctr[mine])
    # per-destination order
    for d, (recv, origin, order, offsets) in enumerate(results):
        rec = recv.cpu().numpy().view(RECORD_DTYPE).ravel() if recv.shape[0] else np.zeros(0, RECORD_DTYPE)
        offs = offsets.cpu().numpy().view(np.uint32)
        ordr = order.cpu().numpy().view(np.uint32)
        glob = np.array([ranks[origin[k]]["sel"][rec["packet"][k]] for k in range(len(rec))], np.int64)
        for slot, h in enumerate(part.hosts_of[d]):
            got = glob[ordr[offs[slot]:offs[slot + 1]]]
            exp = want["dst_order"][want["dst_offsets"][h]:want["dst_offsets"][h + 1]]
            assert np.array_equal(got, exp), (d, h)
        assert np.array_equal(rec["event_id"], want["event_id"][glob])
        assert np.array_equal(rec["deliver_time_ns"], want["deliver_time"][glob])
    return want


@pytest.mark.parametrize("W", [1, 2, 3, 8])
def test_sharded_round_matches_single(oracle, ctx, W):
    want = _run(oracle, ctx, W, 30000)
    assert want["delivered"] > 0


def test_sharded_round_with_rng_skip(oracle, ctx):
    """Other RNG consumers' steps (sg_packets.rng_skip) on the sharded source phase."""
    want = _run(oracle, ctx, 3, 30000, skip=True)
    assert want["delivered"] > 0


@pytest.mark.parametrize("n_packets", [150000, 600000])
def test_sharded_wave_sorted_slots(oracle, ctx, n_packets):
    """About 100 and 400 received records per destination: order-keyed slots sorted by
    one wave each in registers ((time, order key) pairs, 2 keys per lane), and by the block
    past 256."""
    want = _run(oracle, ctx, 2, n_packets, seed=8)
    assert 64 < np.median(np.diff(want["dst_offsets"])) < 512


@pytest.mark.parametrize("p_hot", [0.0, 0.1])
def test_sharded_two_level_bucketing(oracle, ctx, monkeypatch, p_hot):
    """The destination phase's two-level scatter on received records (order keys carried)."""
    monkeypatch.setenv("SG_BUCKET_TWO_LEVEL", "1")
    want = _run(oracle, ctx, 2, 60000, hot=17 if p_hot else -1, seed=6, p_hot=p_hot)
    assert want["delivered"] > 0


@pytest.mark.parametrize("p_hot", [0.1, 0.01])
def test_sharded_hot_destination(oracle, ctx, p_hot):
    # 0.1: the hot slot overfills its region (scan-path fallback); 0.01: a big
    # slot sorted inside the region path's block
    want = _run(oracle, ctx, 4, 120000, hot=17, seed=5, p_hot=p_hot)
    assert np.diff(want["dst_offsets"]).max() > 100


@pytest.mark.parametrize("W,cap_scale", [(2, 1.3), (4, 1.3), (3, 0.5)])
def test_padded_exchange_matches_single(oracle, ctx, W, cap_scale):
    """sg_deliver_source_padded / sg_deliver_bucket_padded: every rank's records for
    rank d in a block of `cap` slots, exchanged by concatenating block d of every
    sender (what the equal-split all-to-all does), bucketed with one sync; the same
    per-destination order, statuses and global stats as one oracle round.  cap_scale
    0.5: blocks too small, so pair_max > cap, and the round is exchanged again exactly
    (sg_deliver_pad_to_compact + sg_deliver_bucket)."""
    import torch

    from shadow_amd.dist import exchange_padded, gpu_bucket_phase_padded, gpu_pad_to_compact, \
        gpu_source_phase_padded, _records_all_to_all

    lat, loss, hosts = _world(oracle, seed=7)
    nu = lat.shape[0]
    part = HostPartition(hosts["route"], nu, W)
    start, end = T0 + 10**9, T0 + 10**9 + 10**6
    n = 40000
    pk = synth.make_packets(n, hosts, start, end, seed=31, p_unknown_dst=0.01, hot_dst=9, p_hot=0.02)
    owner_of_pkt = part.owner[pk["src"]]
    cap = max(256, int(cap_scale * n / W / W))
    ranks = []
    for r in range(W):
        r0, r1, per = row_range(nu, W, r)
        sel = np.nonzero(owner_of_pkt == r)[0]
        ht = HostTable(hosts["ip"], hosts["route"], hosts["seed"], ctx=ctx)
        dl = torch.from_numpy(np.ascontiguousarray(lat[r0:r1]).view(np.int64).ravel()).cuda()
        df = torch.from_numpy(np.ascontiguousarray(loss[r0:r1]).ravel()).cuda()
        table = DeviceTable(dl, df, nu, r0)
        batch = PacketBatch.from_numpy(pk["src"][sel], pk["dst_ip"][sel], pk["payload"][sel], pk["send_time"][sel])
        sd = ShardedDelivery(ctx, ht, table, part, r, W)
        src = gpu_source_phase_padded(ctx, ht, table, batch, end, 2**63, 0, sd.owner_dev, W, cap)
        ranks.append(dict(sel=sel, sd=sd, src=src, send_padded=src.send_padded.clone(), send=src.send.clone(),
                          xrow=src.xrow.clone(), status=src.status[:len(sel)].cpu().numpy()))
    xall = torch.cat([R["xrow"] for R in ranks])
    xa = xall.cpu().numpy().view(np.uint64).reshape(W, 3 + W)
    rng0 = np.stack([oracle.xoshiro_seed(int(s)) for s in hosts["seed"]]).astype(np.uint64)
    want = oracle.deliver_round(end, 2**63, 0, pk["src"], pk["dst_ip"], pk["payload"], pk["send_time"],
                                hosts["ip"], hosts["route"], lat, loss, rng0, np.zeros(hosts["n"], np.uint64))
    overflow = int(xa[:, 3:].max()) > cap
    assert overflow == (cap_scale < 1)
    sels = [R["sel"] for R in ranks]
    for d, R in enumerate(ranks):
        assert np.array_equal(R["status"], want["status"][R["sel"]])
        recv = torch.cat([S["send_padded"][d * cap:(d + 1) * cap] for S in ranks]).contiguous()
        order, offsets, g, recv_counts, pair_max = gpu_bucket_phase_padded(
            ctx, recv, cap, xall, d, R["sd"].local_dev, len(part.local), part.n_local(d))
        assert g == (want["delivered"], want["min_deliver"], want["min_lat"])
        assert recv_counts == [int(x) for x in xa[:, 3 + d]] and pair_max == int(xa[:, 3:].max())
        if overflow:  # the fallback: compact records, exact exchange by concatenation, exact bucketing
            comp = []
            for S in ranks:
                S["src"].send_padded, S["src"].send, S["src"].xrow = S["send_padded"], S["send"].clone(), S["xrow"]
                full = gpu_pad_to_compact(ctx, S["src"], W)
                sc = [int(x) for x in S["xrow"].cpu().numpy().view(np.uint64)[3:]]
                off = sum(sc[:d])
                comp.append(full[off:off + sc[d]].clone())
            recv = torch.cat(comp).contiguous()
            order, offsets = R["sd"].bucket_fn(ctx, recv, recv.shape[0], R["sd"].local_dev, len(part.local),
                                               part.n_local(d))
            origin = np.repeat(np.arange(W), recv_counts)
        else:
            origin = np.arange(W * cap) // cap
        rec = recv.cpu().numpy().view(RECORD_DTYPE).ravel()
        offs = offsets.cpu().numpy().view(np.uint32)
        ordr = order.cpu().numpy().view(np.uint32)
        for slot, h in enumerate(part.hosts_of[d]):
            ks = ordr[offs[slot]:offs[slot + 1]].astype(np.int64)
            got = np.array([sels[origin[k]][rec["packet"][k]] for k in ks], np.int64)
            exp = want["dst_order"][want["dst_offsets"][h]:want["dst_offsets"][h + 1]]
            assert np.array_equal(got, exp), (d, h)
