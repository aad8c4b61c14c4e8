"""GPU parity: one delivery round (HIP) vs the CPU oracle, bit-exact.

Compares per-packet status (delivered / dropped by loss / unknown destination /
after sim end), deliver time, event id, the destination buckets and their
EventQueue order, the round minima, and the hosts' RNG streams and event-id
counters after the round (so consecutive rounds stay in lockstep).
"""
import os

import numpy as np
import pytest

from shadow_amd import ShadowGpuError, _capi, synth
from shadow_amd.worker import DeviceTable, HostTable, PacketBatch, deliver_round

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


_PACKED = {"on": False}


@pytest.fixture(autouse=True, params=[False, True], ids=["two_array", "path_key"])
def table_form(request):
    """Every round runs twice: gathering (latency, loss) from the two arrays,
    and from the packed path-key table (sg_table_pack)."""
    _PACKED["on"] = request.param
    yield request.param
    _PACKED["on"] = False


def _device_table(lat, loss, row_begin=0):
    import torch

    n_cols = lat.shape[1]
    dl = torch.from_numpy(np.ascontiguousarray(lat).view(np.int64).ravel()).cuda()
    df = torch.from_numpy(np.ascontiguousarray(loss).ravel()).cuda()
    t = DeviceTable(dl, df, n_cols, row_begin)
    if _PACKED["on"]:
        wide = bool((np.asarray(lat, dtype=np.uint64) >> np.uint64(32)).any())
        assert t.pack() == (not wide)
    return t


def _run_both(oracle, ctx, lat, loss, hosts, pk, round_end, sim_end, boot, rng0=None, ctr0=None):
    H = hosts["n"]
    ht = HostTable(hosts["ip"], hosts["route"], hosts["seed"], ctx=ctx)
    if rng0 is not None:
        ht.set_state(rng0, ctr0)
    rng, ctr = ht.get_state()
    want = oracle.deliver_round(round_end, sim_end, boot, pk["src"], pk["dst_ip"], pk["payload"], pk["send_time"],
                                hosts["ip"], hosts["route"], lat, loss, rng, ctr)
    batch = PacketBatch.from_numpy(pk["src"], pk["dst_ip"], pk["payload"], pk["send_time"])
    out = deliver_round(ht, _device_table(lat, loss), batch, round_end, sim_end, boot)
    got = out.to_numpy(len(pk["src"]))
    grng, gctr = ht.get_state()
    return want, got, (rng, ctr), (grng, gctr), ht


def _assert_same(want, got, ost, gst):
    assert np.array_equal(got["status"], want["status"])
    assert np.array_equal(got["deliver_time"], want["deliver_time"])
    assert np.array_equal(got["event_id"], want["event_id"])
    assert np.array_equal(got["dst_offsets"], want["dst_offsets"])
    assert np.array_equal(got["dst_order"], want["dst_order"])
    assert got["delivered"] == want["delivered"]
    assert got["min_deliver"] == want["min_deliver"] and got["min_lat"] == want["min_lat"]
    assert np.array_equal(gst[0], ost[0]) and np.array_equal(gst[1], ost[1])


def test_seeding_matches_seed_from_u64(oracle, ctx):
    hosts = synth.make_hosts(50, 5)
    ht = HostTable(hosts["ip"], hosts["route"], hosts["seed"], ctx=ctx)
    rng, ctr = ht.get_state()
    for h in range(50):
        assert np.array_equal(rng[h], oracle.xoshiro_seed(int(hosts["seed"][h])))
    assert (ctr == 0).all()


def test_golden_round(ctx):
    z = np.load(os.path.join(GOLD, "deliver_small.npz"))
    ht = HostTable(z["host_ip"], z["host_route"], z["host_seed"], ctx=ctx)
    rng, ctr = ht.get_state()
    assert np.array_equal(rng, z["rng0"]) and np.array_equal(ctr, z["ctr0"])
    batch = PacketBatch.from_numpy(z["src"], z["dst_ip"], z["payload"], z["send_time"])
    r = z["round"]
    out = deliver_round(ht, _device_table(z["tab_lat"], z["tab_loss"]), batch, int(r[0]), int(r[1]), int(r[2]))
    got = out.to_numpy(len(z["src"]))
    assert np.array_equal(got["status"], z["status"])
    assert np.array_equal(got["deliver_time"], z["deliver_time"])
    assert np.array_equal(got["event_id"], z["event_id"])
    assert np.array_equal(got["dst_order"], z["dst_order"])
    assert np.array_equal(got["dst_offsets"], z["dst_offsets"])
    assert [got["delivered"], got["min_deliver"], got["min_lat"]] == z["stats"].tolist()
    rng1, ctr1 = ht.get_state()
    assert np.array_equal(rng1, z["rng1"]) and np.array_equal(ctr1, z["ctr1"])


def _world(n_nodes=64, n_hosts=2000, seed=1, lossy=True):
    from oracle import oracle as O

    g = synth.ring_chords_graph(n_nodes, 6.0, seed=seed)
    rc, lat, loss, _ = O.shortest_paths(n_nodes, g["src"], g["dst"], g["lat"], g["loss"], False,
                                        np.arange(n_nodes, dtype=np.uint32), threads=8)
    assert rc == 0
    if lossy:
        loss = loss.copy()
        loss[::2, 1::3] = np.float32(0.3)
        loss[5, :] = np.float32(1.0)
    hosts = synth.make_hosts(n_hosts, n_nodes, general_seed=seed, exact_seeds=n_hosts <= 5000)
    return lat, loss, hosts


T0 = 946684800 * 10**9  # EmulatedTime SIMULATION_START


@pytest.mark.parametrize("seed", [1, 2])
def test_random_round(oracle, ctx, seed):
    lat, loss, hosts = _world(seed=seed)
    start, end = T0 + 10**9, T0 + 10**9 + 10**6
    pk = synth.make_packets(60000, hosts, start, end, seed=seed, p_unknown_dst=0.01)
    pk["send_time"][::997] = end + 5 * 10**8  # some at/after sim end
    want, got, ost, gst, _ = _run_both(oracle, ctx, lat, loss, hosts, pk, end, end + 5 * 10**8, start + 300_000)
    assert want["delivered"] > 0 and (want["status"] == oracle.ST_DROP_LOSS).any()
    _assert_same(want, got, ost, gst)


def test_hot_destination_big_buckets(oracle, ctx):
    """Skewed destinations: buckets far above the small-sort and LDS-chunk sizes."""
    lat, loss, hosts = _world(n_hosts=3000, seed=3)
    start, end = T0 + 2 * 10**9, T0 + 2 * 10**9 + 10**6
    pk = synth.make_packets(200000, hosts, start, end, seed=5, hot_dst=11, p_hot=0.15)
    pk2 = synth.make_packets(200000, hosts, start, end, seed=6, hot_dst=12, p_hot=0.02)
    want, got, ost, gst, _ = _run_both(oracle, ctx, lat, loss, hosts, pk, end, 2**63, 0)
    assert np.diff(want["dst_offsets"]).max() > 20000
    _assert_same(want, got, ost, gst)
    want, got, ost, gst, _ = _run_both(oracle, ctx, lat, loss, hosts, pk2, end, 2**63, 0)
    _assert_same(want, got, ost, gst)
    # a big slot (k_sort_big) whose super-bucket still fits its region (no fallback)
    pk3 = synth.make_packets(200000, hosts, start, end, seed=7, hot_dst=13, p_hot=0.0025)
    want, got, ost, gst, _ = _run_both(oracle, ctx, lat, loss, hosts, pk3, end, 2**63, 0)
    assert 100 < np.diff(want["dst_offsets"]).max() < 2000
    _assert_same(want, got, ost, gst)


@pytest.mark.parametrize("per_dst", [20, 50, 100, 200, 400, 560])
def test_slots_around_inblock_sort_limits(oracle, ctx, per_dst):
    """Entries per destination across the region path's in-block sort classes: rank sort
    up to 32, one wave's register bitonic sort for 33-64, 65-128 and 129-256 (1, 2 and 4
    keys per lane), the block's bitonic sort above 256."""
    lat, loss, hosts = _world(n_hosts=3000, seed=9)
    start, end = T0 + 10**9, T0 + 10**9 + 10**6
    pk = synth.make_packets(per_dst * 3000, hosts, start, end, seed=9 + per_dst)
    want, got, ost, gst, _ = _run_both(oracle, ctx, lat, loss, hosts, pk, end, 2**63, 0)
    sizes = np.diff(want["dst_offsets"])
    lo, hi = sizes.min(), sizes.max()
    assert lo < per_dst < hi
    _assert_same(want, got, ost, gst)


@pytest.mark.parametrize("hot", [False, True])
def test_scan_path_bucketing(oracle, ctx, monkeypatch, hot):
    """SG_BUCKET_REGION=0 forces the histogram + scan bucketing path (the
    region path's fallback) for every round."""
    monkeypatch.setenv("SG_BUCKET_REGION", "0")
    lat, loss, hosts = _world(n_hosts=3000, seed=3)
    start, end = T0 + 2 * 10**9, T0 + 2 * 10**9 + 10**6
    pk = synth.make_packets(100000, hosts, start, end, seed=8, hot_dst=14 if hot else -1, p_hot=0.1 if hot else 0.0)
    want, got, ost, gst, _ = _run_both(oracle, ctx, lat, loss, hosts, pk, end, 2**63, 0)
    _assert_same(want, got, ost, gst)


@pytest.mark.parametrize("hot", [0.0, 0.0025, 0.1, 0.5])
def test_two_level_bucketing(oracle, ctx, monkeypatch, hot):
    """SG_BUCKET_TWO_LEVEL=1 forces the two-level region scatter (coarse buckets,
    then super-buckets; the default from 512 super-buckets on, e.g. C5).  0.1: the
    hot slot overfills its coarse sub-region, and the round falls back to the scan
    path from the second level; 0.5 overfills the coarse level itself.  Consecutive
    rounds alternate with the one-level scatter, so both
    counter parities of both levels are reused."""
    lat, loss, hosts = _world(n_hosts=3000, seed=12)
    ht = HostTable(hosts["ip"], hosts["route"], hosts["seed"], ctx=ctx)
    rng, ctr = ht.get_state()
    tab = _device_table(lat, loss)
    for k in range(5):
        monkeypatch.setenv("SG_BUCKET_TWO_LEVEL", "0" if k == 2 else "1")
        start, end = T0 + k * 10**6, T0 + (k + 1) * 10**6
        pk = synth.make_packets(150000, hosts, start, end, seed=40 + k, hot_dst=7 if hot else -1, p_hot=hot)
        want = oracle.deliver_round(end, 2**63, 0, pk["src"], pk["dst_ip"], pk["payload"], pk["send_time"],
                                    hosts["ip"], hosts["route"], lat, loss, rng, ctr)
        out = deliver_round(ht, tab, PacketBatch.from_numpy(pk["src"], pk["dst_ip"], pk["payload"], pk["send_time"]),
                            end, 2**63, 0)
        _assert_same(want, out.to_numpy(150000), (rng, ctr), ht.get_state())


def test_equal_times_order_by_source(oracle, ctx):
    """All packets clamp to round_end: order falls back to (src_host_id, event id)."""
    lat, loss, hosts = _world(n_hosts=500, seed=4, lossy=False)
    end = T0 + 10**12  # far beyond send + latency -> every deliver time == round_end
    pk = synth.make_packets(20000, hosts, T0, T0 + 1000, seed=7)
    want, got, ost, gst, _ = _run_both(oracle, ctx, lat, loss, hosts, pk, end, 2**63, 0)
    assert (want["deliver_time"][want["status"] == 0] == end).all()
    _assert_same(want, got, ost, gst)


def test_consecutive_rounds_keep_streams(oracle, ctx):
    lat, loss, hosts = _world(n_hosts=800, seed=5)
    ht = HostTable(hosts["ip"], hosts["route"], hosts["seed"], ctx=ctx)
    rng, ctr = ht.get_state()
    tab = _device_table(lat, loss)
    for k in range(3):
        start, end = T0 + k * 10**6, T0 + (k + 1) * 10**6
        pk = synth.make_packets(15000, hosts, start, end, seed=20 + k)
        want = oracle.deliver_round(end, 2**63, 0, pk["src"], pk["dst_ip"], pk["payload"], pk["send_time"],
                                    hosts["ip"], hosts["route"], lat, loss, rng, ctr)
        out = deliver_round(ht, tab, PacketBatch.from_numpy(pk["src"], pk["dst_ip"], pk["payload"], pk["send_time"]),
                            end, 2**63, 0)
        _assert_same(want, out.to_numpy(15000), (rng, ctr), ht.get_state())


def test_interleaved_rng_consumers(oracle, ctx):
    """sg_packets.rng_skip: the source host's other Host::random_mut() consumers
    (getrandom, port choices, host_rngDouble; host.rs:645-647) took rng_skip[i]
    steps before packet i.  Three rounds with skips on every kind of packet
    (delivered, lost, unknown destination, past sim end), then sg_hosts_skip for
    steps no later packet carried (hosts repeated), against the oracle."""
    lat, loss, hosts = _world(n_hosts=800, seed=6)
    ht = HostTable(hosts["ip"], hosts["route"], hosts["seed"], ctx=ctx)
    rng, ctr = ht.get_state()
    tab = _device_table(lat, loss)
    g = np.random.default_rng(17)
    for k in range(3):
        start, end = T0 + k * 10**6, T0 + (k + 1) * 10**6
        pk = synth.make_packets(20000, hosts, start, end, seed=60 + k, p_unknown_dst=0.02)
        sim_end = end + 10**9 if k < 2 else start + 500_000  # the last round crosses sim end
        skip = np.where(g.random(20000) < 0.7, 0, g.integers(1, 6, 20000)).astype(np.uint32)
        skip[::1999] = 300  # a long syscall burst
        want = oracle.deliver_round(end, sim_end, 0, pk["src"], pk["dst_ip"], pk["payload"], pk["send_time"],
                                    hosts["ip"], hosts["route"], lat, loss, rng, ctr, rng_skip=skip)
        out = deliver_round(ht, tab, PacketBatch.from_numpy(pk["src"], pk["dst_ip"], pk["payload"], pk["send_time"],
                                                            rng_skip=skip), end, sim_end, 0)
        _assert_same(want, out.to_numpy(20000), (rng, ctr), ht.get_state())
        assert (want["status"] == oracle.ST_SIM_END).any() == (k == 2)
    ids = np.array([3, 5, 3, 799, 0], np.uint32)
    steps = np.array([2, 1, 4, 10, 1], np.uint64)
    ht.skip(ids, steps)
    for h, n in zip(ids, steps):
        for _ in range(int(n)):
            oracle.xoshiro_next_u64(rng[h])
    grng, gctr = ht.get_state()
    assert np.array_equal(grng, rng) and np.array_equal(gctr, ctr)


def test_edge_cases(oracle, ctx):
    lat, loss, hosts = _world(n_hosts=40, seed=6)
    # empty round
    pk = dict(src=np.zeros(0, np.uint32), dst_ip=np.zeros(0, np.uint32), payload=np.zeros(0, np.uint32),
              send_time=np.zeros(0, np.uint64))
    ht = HostTable(hosts["ip"], hosts["route"], hosts["seed"], ctx=ctx)
    out = deliver_round(ht, _device_table(lat, loss), PacketBatch.from_numpy(**{
        "src_host": pk["src"], "dst_ipv4": pk["dst_ip"], "payload_len": pk["payload"], "send_time_ns": pk["send_time"]}),
        T0 + 10, 2**63, 0)
    assert out.n_delivered == 0 and out.min_deliver_time_ns == 2**64 - 1
    assert (out.dst_offsets.cpu().numpy() == 0).all()
    # a single host sending to itself, all acks, all unknown, all after end
    for kind in ("self", "ack", "unknown", "late"):
        n = 100
        src = np.full(n, 3, np.uint32)
        dst_ip = np.full(n, hosts["ip"][3] if kind == "self" else hosts["ip"][9], np.uint32)
        if kind == "unknown":
            dst_ip[:] = 7
        pay = np.zeros(n, np.uint32) if kind == "ack" else np.full(n, 100, np.uint32)
        t = np.arange(T0, T0 + n, dtype=np.uint64)
        sim_end = T0 if kind == "late" else 2**63
        p = dict(src=src, dst_ip=dst_ip, payload=pay, send_time=t)
        want, got, ost, gst, _ = _run_both(oracle, ctx, lat, loss, hosts, p, T0 + 10**6, sim_end, 0)
        _assert_same(want, got, ost, gst)


def test_unsorted_sources_rejected(ctx):
    lat, loss, hosts = _world(n_hosts=10, seed=7)
    ht = HostTable(hosts["ip"], hosts["route"], hosts["seed"], ctx=ctx)
    b = PacketBatch.from_numpy([2, 1], hosts["ip"][[0, 0]], [1, 1], [T0, T0])
    with pytest.raises(ShadowGpuError) as e:
        deliver_round(ht, _device_table(lat, loss), b, T0 + 10, 2**63, 0)
    assert e.value.code == _capi.SG_ERR_UNSORTED


@pytest.mark.parametrize("kind", ["src_range", "unsorted", "route_range"])
def test_rejected_batch_leaves_hosts_unchanged(oracle, ctx, kind):
    """A rejected batch is all-or-nothing: no host's RNG stream or event counter
    moves, the error flags are cleared for the next round, and the next
    round on the SAME host table is exact."""
    lat, loss, hosts = _world(n_hosts=200, seed=9)
    ht = HostTable(hosts["ip"], hosts["route"], hosts["seed"], ctx=ctx)
    start, end = T0 + 10**9, T0 + 10**9 + 10**6
    # a good round first, so the state is not the seed state
    pk0 = synth.make_packets(2000, hosts, T0, T0 + 10**6, seed=3)
    deliver_round(ht, _device_table(lat, loss), PacketBatch.from_numpy(pk0["src"], pk0["dst_ip"], pk0["payload"],
                                                                    pk0["send_time"]), T0 + 10**6, 2**63, 0)
    rng0, ctr0 = ht.get_state()
    table = _device_table(lat, loss)
    if kind == "src_range":  # hosts 0..4 send, then source 250 (out of range)
        src = np.array([0, 1, 2, 3, 4, 250], np.uint32)
    elif kind == "unsorted":  # 0..4 are well grouped, then host 1 again
        src = np.array([0, 1, 2, 3, 4, 1], np.uint32)
    else:  # a table shard holding rows [0, 5): host 7's route row 7 is outside it
        src = np.array([0, 1, 2, 3, 4, 7], np.uint32)
        keep = hosts["route"] < 5
        assert keep[:5].all() and not keep[7]
        import torch
        table = DeviceTable(torch.from_numpy(np.ascontiguousarray(lat[:5]).view(np.int64).ravel()).cuda(),
                            torch.from_numpy(np.ascontiguousarray(loss[:5]).ravel()).cuda(), lat.shape[1], 0)
    dst = hosts["ip"][(src + 1) % hosts["n"]]
    bad = PacketBatch.from_numpy(src, dst, np.ones(len(src), np.uint32), np.full(len(src), T0 + 2 * 10**6, np.uint64))
    with pytest.raises(ShadowGpuError) as e:
        deliver_round(ht, table, bad, T0 + 3 * 10**6, 2**63, 0)
    assert e.value.code == (_capi.SG_ERR_UNSORTED if kind == "unsorted" else _capi.SG_ERR_INVALID_ARG)
    rng1, ctr1 = ht.get_state()
    assert np.array_equal(rng1, rng0) and np.array_equal(ctr1, ctr0), "a rejected batch changed host state"
    pk = synth.make_packets(3000, hosts, start, end, seed=9)
    want = oracle.deliver_round(end, 2**63, 0, pk["src"], pk["dst_ip"], pk["payload"], pk["send_time"],
                                hosts["ip"], hosts["route"], lat, loss, rng0.copy(), ctr0.copy())
    out = deliver_round(ht, _device_table(lat, loss),
                        PacketBatch.from_numpy(pk["src"], pk["dst_ip"], pk["payload"], pk["send_time"]), end, 2**63, 0)
    got = out.to_numpy(len(pk["src"]))
    for k in ("status", "deliver_time", "event_id", "dst_offsets", "dst_order"):
        assert np.array_equal(got[k], want[k]), k


def test_arrival_time_overflow_is_an_error(oracle, ctx):
    """send time + latency past EMUTIME_MAX (u64::MAX - 1): EmulatedTime + SimulationTime
    panics in the reference (emulated_time.rs:121-126, worker.rs:381); here the call
    fails with SG_ERR_TIME_OVERFLOW and the oracle raises OverflowError."""
    hosts = synth.make_hosts(4, 2)
    lat = np.full((2, 2), 10**6, np.uint64)
    loss = np.zeros((2, 2), np.float32)
    for t_send, bad in ((2**64 - 10**6 - 2, False), (2**64 - 10**6 - 1, True), (2**64 - 10, True)):
        src = np.array([0], np.uint32)
        dst = hosts["ip"][[1]]
        ht = HostTable(hosts["ip"], hosts["route"], hosts["seed"], ctx=ctx)
        rng, ctr = ht.get_state()
        b = PacketBatch.from_numpy(src, dst, [100], np.array([t_send], np.uint64))
        if bad:
            with pytest.raises(OverflowError):
                oracle.deliver_round(0, 2**64 - 1, 0, src, dst, [100], [t_send], hosts["ip"], hosts["route"], lat,
                                     loss, rng, ctr)
            with pytest.raises(ShadowGpuError) as e:
                deliver_round(ht, _device_table(lat, loss), b, 0, 2**64 - 1, 0)
            assert e.value.code == _capi.SG_ERR_TIME_OVERFLOW
        else:
            want = oracle.deliver_round(0, 2**64 - 1, 0, src, dst, [100], [t_send], hosts["ip"], hosts["route"],
                                        lat, loss, rng, ctr)
            got = deliver_round(ht, _device_table(lat, loss), b, 0, 2**64 - 1, 0).to_numpy(1)
            assert int(got["deliver_time"][0]) == int(want["deliver_time"][0]) == 2**64 - 2


@pytest.fixture(scope="module")
def c4_world(ctx):
    """The C4 workload: the 10k-node C3 table built on the GPU once,
    100k hosts (node h mod 10k), 1M packets."""
    import time

    import torch

    from shadow_amd import NetworkGraph

    t0 = time.perf_counter()
    g = synth.ring_chords_graph(10000, 8.0, seed=1)
    net = NetworkGraph(g["n"], g["src"], g["dst"], g["lat"], g["loss"], g["directed"], ctx=ctx)
    n = 10000
    used = np.arange(n, dtype=np.uint32)
    dl = torch.empty(n * n, dtype=torch.int64, device="cuda")
    df = torch.empty(n * n, dtype=torch.float32, device="cuda")
    net.build_rows_device(used, 0, n, dl.data_ptr(), df.data_ptr(), True)
    lat = dl.cpu().numpy().view(np.uint64).reshape(n, n)
    loss = df.cpu().numpy().reshape(n, n)
    del dl, df
    hosts = synth.make_hosts(100000, n, general_seed=1, exact_seeds=True)
    start, end = T0 + 10**9, T0 + 10**9 + 10**6
    pk = synth.make_packets(1_000_000, hosts, start, end, seed=100)
    print(f"[c4_world] built in {time.perf_counter() - t0:.1f} s", flush=True)
    return lat, loss, hosts, pk, end


def test_c4_full_round(oracle, ctx, c4_world):
    """The C4 round at full size: exact against the CPU restatement in every output."""
    import time

    lat, loss, hosts, pk, end = c4_world
    t0 = time.perf_counter()
    want, got, ost, gst, _ = _run_both(oracle, ctx, lat, loss, hosts, pk, end, 2**63, 0)
    print(f"[c4] round + oracle in {time.perf_counter() - t0:.1f} s", flush=True)
    assert want["delivered"] > 700_000
    _assert_same(want, got, ost, gst)


def test_duplicate_ip_rejected(ctx):
    with pytest.raises(ShadowGpuError) as e:
        HostTable([5, 5], [0, 0], [1, 2], ctx=ctx)
    assert e.value.code == _capi.SG_ERR_DUPLICATE_IP


def test_sparse_addresses_use_sorted_lookup(oracle, ctx):
    lat, loss, hosts = _world(n_hosts=300, seed=8)
    hosts["ip"] = (np.random.default_rng(1).permutation(2**20)[:300].astype(np.uint32) * 4000 + 7).astype(np.uint32)
    pk = synth.make_packets(8000, hosts, T0, T0 + 10**6, seed=9, p_unknown_dst=0.05)
    want, got, ost, gst, _ = _run_both(oracle, ctx, lat, loss, hosts, pk, T0 + 10**6, 2**63, 0)
    _assert_same(want, got, ost, gst)


def test_pack_refuses_wide_latency(oracle, ctx):
    """A latency of 2^32 ns or more keeps the two-array form (pack returns False)
    and the round is still exact."""
    rng = np.random.default_rng(7)
    hosts = synth.make_hosts(40, 6)
    lat = rng.integers(1, 1000, size=(6, 6)).astype(np.uint64)
    lat[:, 3] = np.uint64(1) << np.uint64(33)
    loss = (rng.random((6, 6), dtype=np.float32) * 0.3).astype(np.float32)
    t = _device_table(lat, loss)
    assert not t.pack() and t.path_key is None
    start, end = T0 + 10**9, T0 + 10**9 + 10**6
    pk = synth.make_packets(500, hosts, start, end, seed=3)
    want, got, ost, gst, _ = _run_both(oracle, ctx, lat, loss, hosts, pk, end, end + 10**12, 0)
    assert want["delivered"] > 0
    _assert_same(want, got, ost, gst)


def test_c5_packet_count_round(oracle, ctx, table_form):
    """10M packets in one round (the C5 packet count) over 60k hosts: the region
    bucketing runs near its super-bucket limit (3750 of 4096).  The bucketing does
    not see the table form: the packed one only (tests/test_c5_gpu.py runs the
    full-size round on both)."""
    if not table_form:
        pytest.skip("the bucketing is the same for both table forms")
    lat, loss, hosts = _world(n_nodes=500, n_hosts=60000, seed=21)
    start, end = T0 + 10**9, T0 + 10**9 + 10**6
    pk = synth.make_packets(10_000_000, hosts, start, end, seed=21, p_unknown_dst=0.001)
    want, got, ost, gst, _ = _run_both(oracle, ctx, lat, loss, hosts, pk, end, 2**63, 0)
    assert want["delivered"] > 9_000_000
    _assert_same(want, got, ost, gst)


def test_packet_counters(oracle, ctx):
    """RoutingInfo::increment_packet_count on the device (sg_ctx_set_packet_counters,
    graph/mod.rs:451-459, worker.rs:373): one count per delivered packet at its path's cell,
    over two rounds; packets dropped by loss, to unknown addresses or past the end count nothing."""
    import torch

    lat, loss, hosts = _world(seed=4)
    n = lat.shape[0]
    start, end = T0 + 10**9, T0 + 10**9 + 10**6
    counts = torch.zeros(n * n, dtype=torch.int64, device="cuda")
    want = np.zeros(n * n, np.uint64)
    ip_to_host = {int(ip): h for h, ip in enumerate(hosts["ip"])}
    ctx.set_packet_counters(counts)
    try:
        rng0 = ctr0 = None
        for r in range(2):
            pk = synth.make_packets(30000, hosts, start, end, seed=40 + r, p_unknown_dst=0.01)
            pk["send_time"][::501] = end + 5 * 10**8
            w, got, ost, gst, ht = _run_both(oracle, ctx, lat, loss, hosts, pk, end, end + 5 * 10**8, start,
                                             rng0, ctr0)
            _assert_same(w, got, ost, gst)
            rng0, ctr0 = gst
            dlv = np.nonzero(w["status"] == oracle.ST_DELIVERED)[0]
            dh = np.array([ip_to_host[int(x)] for x in pk["dst_ip"][dlv]], np.int64)
            cell = hosts["route"][pk["src"][dlv]].astype(np.int64) * n + hosts["route"][dh].astype(np.int64)
            np.add.at(want, cell, np.uint64(1))
            start, end = end, end + 10**6
        assert want.sum() > 0
        assert np.array_equal(counts.cpu().numpy().view(np.uint64), want)
    finally:
        ctx.set_packet_counters(None)
