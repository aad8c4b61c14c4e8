"""GPU parity of the outbound pipeline (sg_outbound_*: interface fifo ->
relay_inet_out token bucket -> router -> send_packet) against the oracle,
bit-exact: statuses, forward times, event-counter advances, the per-host queue
+ relay state, and the sent batch (send_packet order) -- over consecutive
windows (queued packets and pending tasks carry over); then the sent batch
runs through sg_deliver_round like any round's packets."""
import numpy as np
import pytest

from shadow_amd import ShadowGpuError, _capi, synth
from shadow_amd.router import OutboundPipeline
from shadow_amd.worker import DeviceTable, HostTable, deliver_round

pytestmark = pytest.mark.gpu
T0 = 946684800 * 10**9
MS = 10**6
RKEYS = ("head", "tail", "rflags", "task_time", "task_id", "task_born", "tb_cap", "tb_bal", "tb_inc", "tb_last")


def _dev(a, np_dtype, torch_dtype):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a, dtype=np_dtype).view(torch_dtype)).cuda()


def _sends(hosts, n, t0, t1, seed, p_local=0.05):
    pk = synth.make_packets(n, hosts, t0, t1, seed=seed)
    rng = np.random.default_rng(seed + 1000)
    loc = rng.random(n) < p_local
    dst = np.where(loc, hosts["ip"][pk["src"]], pk["dst_ip"]).astype(np.uint32)
    ln = (pk["payload"] + 40).astype(np.uint32)  # IPv4 + TCP headers
    return pk["src"], pk["send_time"], ln, pk["payload"], dst


def _live_same(got, want):
    """Ring slots still needed: [head - cached, tail) per host."""
    c = want["cap"]
    lo = want["head"].astype(np.int64) - ((want["rflags"] & 4) != 0)
    n = want["tail"].astype(np.int64) - lo
    hh = np.repeat(np.arange(len(n)), n)
    s = lo[hh] + np.arange(int(n.sum())) - np.repeat(np.cumsum(n) - n, n)
    i = hh * c + (s % c)
    for k in ("ring_pkt", "ring_len", "ring_pay", "ring_dst"):
        assert np.array_equal(got[k][i], want[k][i]), k


@pytest.mark.parametrize("bw_mbit,boot_ms,layout", [(1000, 0, ""), (10, 0, ""), (2, 0, ""), (10, 3, ""),
                                                   (2, 0, "1"), (10, 3, "1")])
def test_windows_match_oracle(oracle, ctx, monkeypatch, bw_mbit, boot_ms, layout):
    """2000 hosts, 5 windows of 2 ms, 40k sends each: unthrottled to heavily throttled
    (queues and cached packets carried across windows, tasks pending).  layout "1" forces
    lane-major chunks (sg_codel.hip ChunkMap; ~20 sends per host take contiguous ones)."""
    import torch

    if layout:
        monkeypatch.setenv("SG_LANE_MAJOR", layout)

    H, W, per = 2000, 2 * MS, 40000
    hosts = synth.make_hosts(H, 64, exact_seeds=False)
    rng = np.random.default_rng(bw_mbit + boot_ms)
    bw = rng.integers(bw_mbit * 10**6 // 2, bw_mbit * 10**6 + 1, H).astype(np.uint64)
    ob = OutboundPipeline(hosts["ip"], bw, 1024, ctx=ctx)
    ost = oracle.outbound_state(hosts["ip"], bw, ob.cap)
    n_pk = 5 * per
    fwd_g = torch.full((n_pk,), -1, dtype=torch.int64, device="cuda")
    st_g = torch.zeros(n_pk, dtype=torch.uint8, device="cuda")
    ctr_g = torch.zeros(H, dtype=torch.int64, device="cuda")
    fwd_o, st_o, ctr_o = np.full(n_pk, np.uint64(2**64 - 1)), np.zeros(n_pk, np.uint8), np.zeros(H, np.uint64)
    boot, sim_end = T0 + boot_ms * MS, T0 + 10**12
    total = 0
    for w in range(5):
        t0, t1 = T0 + w * W, T0 + (w + 1) * W
        host, t, ln, pay, dst = _sends(hosts, per, t0, t1, seed=100 * bw_mbit + w)
        pkt = np.arange(w * per, (w + 1) * per, dtype=np.uint32)
        batch, ids = ob.run(_dev(host, np.uint32, np.int32), _dev(t, np.uint64, np.int64),
                            _dev(pkt, np.uint32, np.int32), _dev(ln, np.uint32, np.int32),
                            _dev(pay, np.uint32, np.int32), _dev(dst, np.uint32, np.int32), t1, boot, sim_end,
                            fwd_g, st_g, ctr_g.data_ptr())
        want = oracle.outbound_run(ost, host, t, pkt, ln, pay, dst, t1, boot, sim_end, ctr_o, fwd_o, st_o)
        assert np.array_equal(st_g.cpu().numpy(), st_o)
        m = st_o != 0
        assert np.array_equal(fwd_g.cpu().numpy().view(np.uint64)[m], fwd_o[m])
        assert np.array_equal(ctr_g.cpu().numpy().view(np.uint64), ctr_o)
        assert len(batch) == len(want["packet"])
        assert np.array_equal(batch.src_host.cpu().numpy().view(np.uint32), want["src_host"])
        assert np.array_equal(batch.dst_ipv4.cpu().numpy().view(np.uint32), want["dst_ipv4"])
        assert np.array_equal(batch.payload_len.cpu().numpy().view(np.uint32), want["payload_len"])
        assert np.array_equal(batch.send_time_ns.cpu().numpy().view(np.uint64), want["send_time"])
        assert np.array_equal(ids.cpu().numpy().view(np.uint32), want["packet"])
        got = ob.get_state()
        for k in RKEYS:
            assert np.array_equal(got[k], ost[k]), k
        _live_same(got, ost)
        total += len(want["packet"])
    assert (st_o == 2).any()
    if bw_mbit == 2:
        assert (st_o == 0).any() and (ost["rflags"] & oracle.RL_PENDING).any() and total < n_pk


def _keyed_sends(hosts, n, t0, t1, seed):
    """Sends of which half land exactly on a refill boundary (T0 + k ms, where a blocked
    relay's wake-up falls), each made by a random event: a Packet event (id UINT64_MAX) or a
    Local one created up to 3 ms earlier with a random id.  Per (host, time) the sends are put
    in execution order: Packet events first, then Local ones by (created, id)."""
    host, t, ln, pay, dst = _sends(hosts, n, t0, t1, seed)
    rng = np.random.default_rng(seed + 7)
    snap = rng.random(n) < 0.5
    t = np.where(snap, (t - T0) // MS * MS + T0, t).astype(np.uint64)
    t = np.maximum(t, np.uint64(t0))
    pk = rng.random(n) < 0.2
    born = (t - rng.integers(0, 3 * MS, n).astype(np.uint64)).astype(np.uint64)
    born = np.where(rng.random(n) < 0.3, (born - T0) // MS * MS + T0, born).astype(np.uint64)  # wake births
    eid = rng.integers(0, 5000, n).astype(np.uint64)
    born = np.where(pk, np.uint64(0), born)
    eid = np.where(pk, np.uint64(2**64 - 1), eid)
    o = np.lexsort((eid, born, ~pk, t, host))  # host, time, Packet first, created, id
    return host[o], t[o], ln[o], pay[o], dst[o], eid[o], born[o]


@pytest.mark.parametrize("bw_mbit,layout", [(10, ""), (2, ""), (2, "1")])
def test_same_time_ties_match_oracle(oracle, ctx, monkeypatch, bw_mbit, layout):
    """Wake-ups and sends on the same nanosecond, ordered by the sending event's (created, id)
    against the task's (relay/mod.rs:145-157, event.rs:84-155): 1500 hosts, 4 windows, keyed
    sends (k_outbound<true>) bit-exact with the oracle, task ids included.  The keys must
    matter: the oracle with every Local send created first, and with every one created last,
    disagrees (the ties went both ways)."""
    import torch

    if layout:
        monkeypatch.setenv("SG_LANE_MAJOR", layout)
    H, W, per = 1500, 2 * MS, 30000
    hosts = synth.make_hosts(H, 64, exact_seeds=False)
    bw = np.full(H, bw_mbit * 10**6, np.uint64)
    ob = OutboundPipeline(hosts["ip"], bw, 1024, ctx=ctx)
    ost = oracle.outbound_state(hosts["ip"], bw, ob.cap)
    alt = {k: oracle.outbound_state(hosts["ip"], bw, ob.cap) for k in ("early", "late")}
    n_pk = 4 * per
    fwd_g = torch.full((n_pk,), -1, dtype=torch.int64, device="cuda")
    st_g = torch.zeros(n_pk, dtype=torch.uint8, device="cuda")
    ctr_g = torch.zeros(H, dtype=torch.int64, device="cuda")
    fwd_o, st_o, ctr_o = np.full(n_pk, np.uint64(2**64 - 1)), np.zeros(n_pk, np.uint8), np.zeros(H, np.uint64)
    ctr_alt = {k: np.zeros(H, np.uint64) for k in alt}
    sim_end = T0 + 10**12
    for w in range(4):
        t0, t1 = T0 + w * W, T0 + (w + 1) * W
        host, t, ln, pay, dst, eid, born = _keyed_sends(hosts, per, t0, t1, seed=50 * bw_mbit + w)
        pkt = np.arange(w * per, (w + 1) * per, dtype=np.uint32)
        batch, ids = ob.run(_dev(host, np.uint32, np.int32), _dev(t, np.uint64, np.int64),
                            _dev(pkt, np.uint32, np.int32), _dev(ln, np.uint32, np.int32),
                            _dev(pay, np.uint32, np.int32), _dev(dst, np.uint32, np.int32), t1, 0, sim_end,
                            fwd_g, st_g, ctr_g.data_ptr(), event_id=_dev(eid, np.uint64, np.int64),
                            event_created_ns=_dev(born, np.uint64, np.int64))
        want = oracle.outbound_run(ost, host, t, pkt, ln, pay, dst, t1, 0, sim_end, ctr_o, fwd_o, st_o,
                                   event_id=eid, event_created=born)
        assert np.array_equal(st_g.cpu().numpy(), st_o)
        m = st_o != 0
        assert np.array_equal(fwd_g.cpu().numpy().view(np.uint64)[m], fwd_o[m])
        assert np.array_equal(ctr_g.cpu().numpy().view(np.uint64), ctr_o)
        assert np.array_equal(ids.cpu().numpy().view(np.uint32), want["packet"])
        assert np.array_equal(batch.send_time_ns.cpu().numpy().view(np.uint64), want["send_time"])
        got = ob.get_state()
        for k in RKEYS:
            assert np.array_equal(got[k], ost[k]), k
        _live_same(got, ost)
        scratch = lambda: (np.zeros(n_pk, np.uint64), np.zeros(n_pk, np.uint8))
        for k, shift in (("early", -10**12), ("late", 10**12)):  # every Local send created first / last
            b2 = np.where(eid == np.uint64(2**64 - 1), born, (born.astype(np.int64) + shift).astype(np.uint64))
            oracle.outbound_run(alt[k], host, t, pkt, ln, pay, dst, t1, 0, sim_end, ctr_alt[k], *scratch(),
                                event_id=eid, event_created=b2)
    for k in alt:  # the ties went both ways
        assert not np.array_equal(ctr_alt[k], ctr_o), k


def test_keyed_send_errors(ctx):
    import torch

    ob = OutboundPipeline(np.array([10], np.uint32), np.array([10**9], np.uint64), 16, ctx=ctx)
    f = torch.zeros(8, dtype=torch.int64, device="cuda")
    s = torch.zeros(8, dtype=torch.uint8, device="cuda")
    ctr = torch.zeros(1, dtype=torch.int64, device="cuda")
    args = [_dev([0, 0], np.uint32, np.int32), _dev([T0 + 1, T0 + 1], np.uint64, np.int64),
            _dev([0, 1], np.uint32, np.int32), _dev([100] * 2, np.uint32, np.int32),
            _dev([60] * 2, np.uint32, np.int32), _dev([11, 11], np.uint32, np.int32)]
    born = _dev([T0, T0], np.uint64, np.int64)
    with pytest.raises(ShadowGpuError) as e:  # Local events out of id order at one time
        ob.run(*args, T0 + MS, 0, T0 + 10**12, f, s, ctr.data_ptr(), event_id=_dev([9, 5], np.uint64, np.int64),
               event_created_ns=born)
    assert e.value.code == _capi.SG_ERR_UNSORTED
    with pytest.raises(ShadowGpuError) as e:  # keys need the hosts' counters
        ob.run(*args, T0 + MS, 0, T0 + 10**12, f, s, None, event_id=_dev([5, 9], np.uint64, np.int64),
               event_created_ns=born)
    assert e.value.code == _capi.SG_ERR_INVALID_ARG


def test_sent_batch_feeds_delivery(oracle, ctx):
    """Outbound window -> sg_deliver_round on the sent batch, against the oracle chain."""
    import torch

    from test_deliver_gpu import _world

    lat, loss, hosts = _world(n_hosts=1500, seed=4)
    H = hosts["n"]
    bw = np.full(H, 20 * 10**6, np.uint64)
    start, end = T0 + 10**9, T0 + 10**9 + MS
    host, t, ln, pay, dst = _sends(hosts, 30000, start, end, seed=7)
    pkt = np.arange(len(host), dtype=np.uint32)
    ob = OutboundPipeline(hosts["ip"], bw, 256, ctx=ctx)
    ost = oracle.outbound_state(hosts["ip"], bw, ob.cap)
    fwd_g = torch.zeros(len(pkt), dtype=torch.int64, device="cuda")
    st_g = torch.zeros(len(pkt), dtype=torch.uint8, device="cuda")
    ht = HostTable(hosts["ip"], hosts["route"], hosts["seed"], ctx=ctx)
    rng0, ctr0 = ht.get_state()
    ctr_o = ctr0.copy()
    batch, ids = ob.run(_dev(host, np.uint32, np.int32), _dev(t, np.uint64, np.int64), _dev(pkt, np.uint32, np.int32),
                        _dev(ln, np.uint32, np.int32), _dev(pay, np.uint32, np.int32), _dev(dst, np.uint32, np.int32),
                        end, 0, end + 10**9, fwd_g, st_g, _capi.load().sg_hosts_event_ctr(ht.handle))
    sent = oracle.outbound_run(ost, host, t, pkt, ln, pay, dst, end, 0, end + 10**9, ctr_o,
                               np.zeros(len(pkt), np.uint64), np.zeros(len(pkt), np.uint8))
    lat_t = torch.from_numpy(np.ascontiguousarray(lat).view(np.int64).ravel()).cuda()
    table = DeviceTable(lat_t, torch.from_numpy(np.ascontiguousarray(loss).ravel()).cuda(), lat.shape[1])
    assert table.pack()
    out = deliver_round(ht, table, batch, end, end + 10**9, 0)
    got = out.to_numpy(len(batch))
    want = oracle.deliver_round(end, end + 10**9, 0, sent["src_host"], sent["dst_ipv4"], sent["payload_len"],
                                sent["send_time"], hosts["ip"], hosts["route"], lat, loss, rng0, ctr_o)
    for k in ("status", "deliver_time", "event_id", "dst_offsets", "dst_order"):
        assert np.array_equal(got[k], want[k]), k
    grng, gctr = ht.get_state()
    assert np.array_equal(grng, rng0) and np.array_equal(gctr, ctr_o)
    assert want["delivered"] > 0 and len(batch) < len(pkt)


def test_sent_capacity_and_order_errors(ctx):
    import torch

    ob = OutboundPipeline(np.array([10, 11], np.uint32), np.array([10**9, 10**9], np.uint64), 16, ctx=ctx)
    f = torch.zeros(8, dtype=torch.int64, device="cuda")
    s = torch.zeros(8, dtype=torch.uint8, device="cuda")
    args = [_dev([0, 0, 1], np.uint32, np.int32), _dev([T0 + 1, T0 + 2, T0 + 1], np.uint64, np.int64),
            _dev([0, 1, 2], np.uint32, np.int32), _dev([100] * 3, np.uint32, np.int32),
            _dev([60] * 3, np.uint32, np.int32), _dev([11, 11, 10], np.uint32, np.int32)]
    with pytest.raises(ShadowGpuError) as e:
        ob.run(*args, T0 + MS, 0, T0 + 10**12, f, s, sent_cap=2)
    assert e.value.code == _capi.SG_ERR_CAPACITY
    ob = OutboundPipeline(np.array([10, 11], np.uint32), np.array([10**9, 10**9], np.uint64), 16, ctx=ctx)
    args[1] = _dev([T0 + 2, T0 + 1, T0 + 1], np.uint64, np.int64)
    with pytest.raises(ShadowGpuError) as e:
        ob.run(*args, T0 + MS, 0, T0 + 10**12, f, s)
    assert e.value.code == _capi.SG_ERR_UNSORTED


def test_groups_locals_and_long_hosts(oracle, ctx):
    """Sends on a microsecond grid (same-time groups: one task and id each), local
    sends between non-local ones (no tokens; the bucket's refill time stays at the
    last non-local send), hosts with thousands of sends across chunks, a bootstrap
    boundary inside a window, and a few slow relays that block beside unthrottled
    ones; three windows."""
    import torch

    H = 1500
    hosts = synth.make_hosts(H, 64, exact_seeds=False)
    rng = np.random.default_rng(77)
    bw = np.where(rng.random(H) < 0.05, 2 * 10**6, 10**9).astype(np.uint64)
    ob = OutboundPipeline(hosts["ip"], bw, 8192, ctx=ctx)
    ost = oracle.outbound_state(hosts["ip"], bw, ob.cap)
    per = 30000
    n_pk = 3 * (per + 5000)
    fwd_g = torch.full((n_pk,), -1, dtype=torch.int64, device="cuda")
    st_g = torch.zeros(n_pk, dtype=torch.uint8, device="cuda")
    ctr_g = torch.zeros(H, dtype=torch.int64, device="cuda")
    fwd_o, st_o, ctr_o = np.full(n_pk, np.uint64(2**64 - 1)), np.zeros(n_pk, np.uint8), np.zeros(H, np.uint64)
    boot, sim_end = T0 + 25 * MS, T0 + 10**12
    p0 = 0
    for w in range(3):
        t0, t1 = T0 + w * 20 * MS, T0 + (w + 1) * 20 * MS
        host, t, ln, pay, dst = _sends(hosts, per, t0, t1 - 1000, seed=900 + w, p_local=0.15)
        # two long hosts (several chunks each), times on a 1-us grid
        host = np.r_[host, np.full(2000, 3, np.uint32), np.full(3000, 900, np.uint32)].astype(np.uint32)
        t = np.r_[t, rng.integers(t0, t1 - 1000, 5000).astype(np.uint64)]
        ln = np.r_[ln, rng.integers(40, 1500, 5000).astype(np.uint32)]
        pay = np.r_[pay, np.full(5000, 100, np.uint32)]
        dst = np.r_[dst, np.where(rng.random(5000) < 0.1, hosts["ip"][host[-5000:]], hosts["ip"][(host[-5000:] + 1) % H])]
        t = (t // 1000 * 1000).astype(np.uint64)
        o = np.lexsort((t, host))
        host, t, ln, pay, dst = host[o], t[o], ln[o], pay[o], dst[o].astype(np.uint32)
        pkt = np.arange(p0, p0 + len(host), dtype=np.uint32)
        p0 += len(host)
        batch, ids = ob.run(_dev(host, np.uint32, np.int32), _dev(t, np.uint64, np.int64),
                            _dev(pkt, np.uint32, np.int32), _dev(ln, np.uint32, np.int32),
                            _dev(pay, np.uint32, np.int32), _dev(dst, np.uint32, np.int32), t1, boot, sim_end,
                            fwd_g, st_g, ctr_g.data_ptr())
        want = oracle.outbound_run(ost, host, t, pkt, ln, pay, dst, t1, boot, sim_end, ctr_o, fwd_o, st_o)
        assert np.array_equal(st_g.cpu().numpy(), st_o)
        m = st_o != 0
        assert np.array_equal(fwd_g.cpu().numpy().view(np.uint64)[m], fwd_o[m])
        assert np.array_equal(ctr_g.cpu().numpy().view(np.uint64), ctr_o)
        assert np.array_equal(ids.cpu().numpy().view(np.uint32), want["packet"])
        assert np.array_equal(batch.send_time_ns.cpu().numpy().view(np.uint64), want["send_time"])
        got = ob.get_state()
        for k in RKEYS:
            assert np.array_equal(got[k], ost[k]), k
        _live_same(got, ost)
    assert (st_o == 3).any() or (st_o == 2).any()



def test_tie_task_after_later_event_and_equal_key(oracle, ctx):
    """The hand cases of test_outbound_cpu.py on k_outbound<true>: a wake-up that runs at a
    tie after a later-numbered sending event was created reschedules itself past that id
    (the counter steps before the task, not after it); a send carrying the pending wake-up's
    own key is refused (SG_ERR_UNSORTED), as the oracle refuses it (-6)."""
    import torch

    def go(sends, keys, window_end):
        n = len(sends)
        ob = OutboundPipeline(np.array([10], np.uint32), np.array([8 * 10**6], np.uint64), 8, ctx=ctx)
        f = torch.full((n,), -1, dtype=torch.int64, device="cuda")
        s = torch.zeros(n, dtype=torch.uint8, device="cuda")
        ctr = torch.full((1,), 100, dtype=torch.int64, device="cuda")
        _, ids = ob.run(_dev([0] * n, np.uint32, np.int32), _dev([x[0] for x in sends], np.uint64, np.int64),
                        _dev([x[1] for x in sends], np.uint32, np.int32), _dev([1500] * n, np.uint32, np.int32),
                        _dev([1472] * n, np.uint32, np.int32), _dev([11] * n, np.uint32, np.int32),
                        window_end, 0, T0 + 10**12, f, s, ctr.data_ptr(),
                        event_id=_dev([k[1] for k in keys], np.uint64, np.int64),
                        event_created_ns=_dev([k[0] for k in keys], np.uint64, np.int64))
        return ob.get_state(), ids.cpu().numpy(), s.cpu().numpy(), int(ctr[0])

    st, ids, s, ctr = go([(T0 + 1, 0), (T0 + 1, 1), (T0 + 1, 3), (T0 + MS, 2)], [(T0, 5)] * 3 + [(T0 + 1, 150)],
                         T0 + MS + 1)
    assert list(ids) == [0, 1] and list(s) == [1, 1, 0, 0]
    assert st["task_id"][0] == 151 and st["task_born"][0] == T0 + MS and ctr == 152
    with pytest.raises(ShadowGpuError) as e:  # C made by the wake-up's own key (T0+1, 101)
        go([(T0 + 1, 0), (T0 + 1, 1), (T0 + MS, 2)], [(T0, 5), (T0, 5), (T0 + 1, 101)], T0 + 10 * MS)
    assert e.value.code == _capi.SG_ERR_UNSORTED
    go([(T0 + 1, 0), (T0 + 1, 1), (T0 + MS, 2)], [(T0, 5), (T0, 5), (T0 + 1, 102)], T0 + 10 * MS)


def test_without_sent_batch(ctx):
    """sg_outbound_run with sent = NULL (no sent batch: the window's sums alone, k_codel_reduce)
    gives the same statuses, forward times, event counters, queue and relay state and sent count
    as with one (the offsets and sums in one launch, then the compaction), over three windows."""
    import torch

    H, W, per = 500, 2 * MS, 8000
    hosts = synth.make_hosts(H, 64, exact_seeds=False)
    bw = np.random.default_rng(5).integers(2 * 10**6, 10 * 10**6, H).astype(np.uint64)
    obs = [OutboundPipeline(hosts["ip"], bw, 512, ctx=ctx) for _ in range(2)]
    n_pk = 3 * per
    out = [(torch.full((n_pk,), -1, dtype=torch.int64, device="cuda"), torch.zeros(n_pk, dtype=torch.uint8, device="cuda"),
            torch.zeros(H, dtype=torch.int64, device="cuda")) for _ in range(2)]
    for w in range(3):
        t0, t1 = T0 + w * W, T0 + (w + 1) * W
        host, t, ln, pay, dst = _sends(hosts, per, t0, t1, seed=900 + w)
        pkt = np.arange(w * per, (w + 1) * per, dtype=np.uint32)
        args = (_dev(host, np.uint32, np.int32), _dev(t, np.uint64, np.int64), _dev(pkt, np.uint32, np.int32),
                _dev(ln, np.uint32, np.int32), _dev(pay, np.uint32, np.int32), _dev(dst, np.uint32, np.int32),
                t1, T0, T0 + 10**12)
        batch, _ = obs[0].run(*args, out[0][0], out[0][1], out[0][2].data_ptr())
        none, n_sent = obs[1].run(*args, out[1][0], out[1][1], out[1][2].data_ptr(), collect=False)
        assert none is None and n_sent == len(batch)
        for a, b in zip(out[0], out[1]):
            assert torch.equal(a, b)
        sa, sb = obs[0].get_state(), obs[1].get_state()
        for k in RKEYS:
            assert np.array_equal(sa[k], sb[k]), k
