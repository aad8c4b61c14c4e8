"""GPU parity of the inbound pipeline (sg_inbound_*: router CoDel queue ->
relay_inet_in token bucket) against the oracle, bit-exact: forward times,
statuses, event-counter advances and the whole per-host queue + relay state,
over consecutive windows (pending forward tasks carry over)."""
import numpy as np
import pytest

from shadow_amd import ShadowGpuError, _capi
from shadow_amd.router import InboundPipeline

pytestmark = pytest.mark.gpu
T0 = 946684800 * 10**9
MS = 10**6
QKEYS = ("flags", "interval_end", "drop_next", "cur", "prev", "bytes", "head", "tail")
RKEYS = ("rflags", "task_time", "tb_cap", "tb_bal", "tb_inc", "tb_last")


def _dev(a, np_dtype, torch_dtype):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a, dtype=np_dtype).view(torch_dtype)).cuda()


def _arrivals(rng, H, n, t0, t1):
    host = np.sort(rng.integers(0, H, n)).astype(np.uint32)
    t = np.sort(rng.integers(t0, t1, n)).astype(np.uint64)
    order = np.lexsort((t, host))  # per host ascending time (EventQueue order by time)
    host, t = host[order], t[order]
    ln = rng.choice(np.array([28, 1476, 600], np.uint32), n)
    return host, t, ln


def _live_ring_same(got, want):
    """The queued elements (head .. tail of each host's ring) hold the same packets: an
    ordered call stores arrival indices while it runs and must leave packet ids behind."""
    cap = want["cap"]
    for h in np.nonzero(want["tail"] != want["head"])[0]:
        pos = (np.arange(int(want["head"][h]), int(want["tail"][h]), dtype=np.uint64) % cap).astype(np.int64) + h * cap
        for k in ("ring_pkt", "ring_len", "ring_ts"):
            assert np.array_equal(got[k][pos], want[k][pos]), (k, h)


def _run(ib, ordered, host, t, pkt, ln, wend, boot, sim_end, fwd_g, st_g, ctr_ptr=None):
    """One window through run() or run_ordered(); the ordered call's per-arrival fates are
    scattered to packet ids here (into fwd_g / st_g), so both compare with the oracle alike."""
    import torch

    args = (_dev(host, np.uint32, np.int32), _dev(t, np.uint64, np.int64), _dev(pkt, np.uint32, np.int32),
            _dev(ln, np.uint32, np.int32), wend, boot, sim_end)
    if not ordered:
        return ib.run(*args, fwd_g, st_g, ctr_ptr)
    n = len(host)
    a_st = torch.zeros(max(n, 1), dtype=torch.uint8, device="cuda")
    a_fwd = torch.full((max(n, 1),), -1, dtype=torch.int64, device="cuda")
    before = st_g.clone()
    nd = ib.run_ordered(*args, fwd_g, st_g, a_fwd, a_st, ctr_ptr)
    if n:
        # this call's arrivals are never written by packet id
        p = torch.from_numpy(np.asarray(pkt, np.int64)).cuda()
        assert torch.equal(st_g[p], before[p])
        left = a_st[:n] != 0
        st_g[p[left]] = a_st[:n][left]
        fw = left & (a_st[:n] == 1)
        fwd_g[p[fw]] = a_fwd[:n][fw]
        assert bool((a_fwd[:n][~fw] == -1).all())  # untouched unless forwarded
    return nd


def _same(O, got, want):
    for k in QKEYS + RKEYS:
        assert np.array_equal(got[k], want[k]), k
    # cached packets only where a packet is cached
    m = (want["rflags"] & O.RL_CACHED) != 0
    assert np.array_equal(got["cached_pkt"][m], want["cached_pkt"][m])
    assert np.array_equal(got["cached_len"][m], want["cached_len"][m])


@pytest.mark.parametrize("bw_mbit,boot_ms,layout,ordered", [
    (1000, 0, "", False), (10, 0, "", False), (1, 0, "", False), (10, 40, "", False), (1, 0, "0", False),
    (10, 40, "0", False), (1000, 0, "", True), (1, 0, "", True), (10, 40, "", True), (1, 0, "0", True),
    (10, 40, "0", True)])
def test_windows_match_oracle(oracle, ctx, monkeypatch, bw_mbit, boot_ms, layout, ordered):
    """300 hosts, 5 windows of 60 ms, 60k arrivals: from unthrottled to heavily
    throttled (standing queues, CoDel drop mode, tasks pending across windows).  ~40
    arrivals per host: lane-major chunks by default (sg_codel.hip ChunkMap); layout "0"
    forces contiguous ones.  ordered: sg_inbound_run_ordered (fates in arrival order;
    packets carried from earlier windows by id), the queued rings checked too."""
    import torch

    if layout:
        monkeypatch.setenv("SG_LANE_MAJOR", layout)

    rng = np.random.default_rng(bw_mbit + boot_ms)
    H, W, per = 300, 60 * MS, 12000
    bw = rng.integers(bw_mbit * 10**6 // 2, bw_mbit * 10**6 + 1, H).astype(np.uint64)
    ib = InboundPipeline(bw, 4096, ctx=ctx)
    ost = oracle.inbound_state(bw, ib.cap)
    n_pk = 5 * per
    fwd_g = torch.full((n_pk,), -1, dtype=torch.int64, device="cuda")
    st_g = torch.zeros(n_pk, dtype=torch.uint8, device="cuda")
    ctr_g = torch.zeros(H, dtype=torch.int64, device="cuda")
    fwd_o = np.full(n_pk, np.uint64(2**64 - 1))
    st_o = np.zeros(n_pk, np.uint8)
    ctr_o = np.zeros(H, np.uint64)
    boot, sim_end = T0 + boot_ms * MS, T0 + 10**12
    for w in range(5):
        t0, t1 = T0 + w * W, T0 + (w + 1) * W
        host, t, ln = _arrivals(rng, H, per, t0, t1)
        pkt = np.arange(w * per, (w + 1) * per, dtype=np.uint32)
        nd = _run(ib, ordered, host, t, pkt, ln, t1, boot, sim_end, fwd_g, st_g, ctr_g.data_ptr())
        before = int((st_o == 2).sum())
        oracle.inbound_run(ost, host, t, pkt, ln, t1, boot, sim_end, ctr_o, fwd_o, st_o)
        assert nd == int((st_o == 2).sum()) - before
        assert np.array_equal(st_g.cpu().numpy(), st_o)
        assert np.array_equal(fwd_g.cpu().numpy().view(np.uint64)[st_o == 1], fwd_o[st_o == 1])
        assert np.array_equal(ctr_g.cpu().numpy().view(np.uint64), ctr_o)
        got = ib.get_state()
        _same(oracle, got, ost)
        if ordered:
            _live_ring_same(got, ost)
        for k in ("task_id", "task_born"):
            assert np.array_equal(got[k], ost[k]), k
    if bw_mbit == 1:
        assert (st_o == 2).any() and (ost["rflags"] & oracle.RL_PENDING).any()


def test_empty_window_runs_pending_tasks(oracle, ctx):
    """A window with no arrivals still runs the forward tasks that fall inside it."""
    import torch

    bw = np.array([8000, 8000], np.uint64)  # 1 B per ms
    ib = InboundPipeline(bw, 64, ctx=ctx)
    ost = oracle.inbound_state(bw, ib.cap)
    fwd_g = torch.full((8,), -1, dtype=torch.int64, device="cuda")
    st_g = torch.zeros(8, dtype=torch.uint8, device="cuda")
    fwd_o, st_o, ctr_o = np.full(8, np.uint64(2**64 - 1)), np.zeros(8, np.uint8), np.zeros(2, np.uint64)
    host, t, pkt, ln = [0, 0, 1], [T0 + 5 * MS] * 3, [0, 1, 2], [1500, 1500, 1500]
    args = lambda: (_dev(host, np.uint32, np.int32), _dev(t, np.uint64, np.int64), _dev(pkt, np.uint32, np.int32),
                    _dev(ln, np.uint32, np.int32))
    ib.run(*args(), T0 + 10 * MS, 0, T0 + 10**12, fwd_g, st_g)
    oracle.inbound_run(ost, host, t, pkt, ln, T0 + 10 * MS, 0, T0 + 10**12, ctr_o, fwd_o, st_o)
    e = [_dev([], np.uint32, np.int32), _dev([], np.uint64, np.int64), _dev([], np.uint32, np.int32),
         _dev([], np.uint32, np.int32)]
    ib.run(*e, T0 + 3000 * MS, 0, T0 + 10**12, fwd_g, st_g)
    oracle.inbound_run(ost, [], [], [], [], T0 + 3000 * MS, 0, T0 + 10**12, ctr_o, fwd_o, st_o)
    assert np.array_equal(st_g.cpu().numpy(), st_o) and st_o[1] == 1
    assert np.array_equal(fwd_g.cpu().numpy().view(np.uint64)[st_o == 1], fwd_o[st_o == 1])
    _same(oracle, ib.get_state(), ost)


def test_arrival_after_window_rejected(ctx):
    import torch

    ib = InboundPipeline(np.array([10**9], np.uint64), 16, ctx=ctx)
    with pytest.raises(ShadowGpuError) as e:
        ib.run(_dev([0], np.uint32, np.int32), _dev([T0 + 20 * MS], np.uint64, np.int64),
               _dev([0], np.uint32, np.int32), _dev([100], np.uint32, np.int32), T0 + 10 * MS, 0, T0 + 10**12,
               torch.zeros(4, dtype=torch.int64, device="cuda"), torch.zeros(4, dtype=torch.uint8, device="cuda"))
    assert e.value.code == _capi.SG_ERR_INVALID_ARG


def _run_windows(oracle, ctx, bw, cap, windows, boot, sim_end=T0 + 10**12, ordered=False):
    """Consecutive windows (host, t, ln, window_end) on the GPU and the oracle,
    everything compared after each (statuses, forward times, counters, state, ids)."""
    import torch

    H = len(bw)
    ib = InboundPipeline(bw, cap, ctx=ctx)
    ost = oracle.inbound_state(bw, ib.cap)
    n_pk = sum(len(w[0]) for w in windows)
    fwd_g = torch.full((max(n_pk, 1),), -1, dtype=torch.int64, device="cuda")
    st_g = torch.zeros(max(n_pk, 1), dtype=torch.uint8, device="cuda")
    ctr_g = torch.zeros(H, dtype=torch.int64, device="cuda")
    fwd_o = np.full(max(n_pk, 1), np.uint64(2**64 - 1))
    st_o = np.zeros(max(n_pk, 1), np.uint8)
    ctr_o = np.zeros(H, np.uint64)
    p0 = 0
    for host, t, ln, wend in windows:
        pkt = np.arange(p0, p0 + len(host), dtype=np.uint32)
        p0 += len(host)
        _run(ib, ordered, host, t, pkt, ln, wend, boot, sim_end, fwd_g, st_g, ctr_g.data_ptr())
        oracle.inbound_run(ost, host, t, pkt, ln, wend, boot, sim_end, ctr_o, fwd_o, st_o)
        assert np.array_equal(st_g.cpu().numpy(), st_o)
        assert np.array_equal(fwd_g.cpu().numpy().view(np.uint64)[st_o == 1], fwd_o[st_o == 1])
        assert np.array_equal(ctr_g.cpu().numpy().view(np.uint64), ctr_o)
        got = ib.get_state()
        _same(oracle, got, ost)
        if ordered:
            _live_ring_same(got, ost)
        for k in ("task_id", "task_born"):
            assert np.array_equal(got[k], ost[k]), k
    return st_o, ost


@pytest.mark.parametrize("ordered", [False, True])
def test_groups_chunks_and_slow_relays(oracle, ctx, ordered):
    """Same-time groups of arrivals (a task per group, one id each), long hosts
    crossing chunk boundaries with same-time runs across them, a bootstrap boundary
    inside a window, bucket refills across many intervals, and throttled hosts
    beside unthrottled ones in every block; three windows."""
    rng = np.random.default_rng(41)
    H = 3000
    bw = np.where(rng.random(H) < 0.05, 2 * 10**6, 10**9).astype(np.uint64)  # a few slow relays
    windows = []
    for w in range(3):
        t0, t1 = T0 + w * 20 * MS, T0 + (w + 1) * 20 * MS
        host = np.sort(rng.integers(0, H, 30000)).astype(np.uint32)
        # hosts 5, 700 and 1500 get long runs (several chunks), with same-time runs
        host = np.sort(np.r_[host, np.full(2500, 5), np.full(1800, 700), np.full(3000, 1500)].astype(np.uint32))
        t = np.zeros(len(host), np.uint64)
        for h in np.unique(host):
            idx = np.nonzero(host == h)[0]
            # integer-us times: same-time groups are common; runs of 40 at host 5, 150 at host 1500
            tt = np.sort(rng.integers(t0, t1 - 1000, len(idx)) // 1000 * 1000)
            if h == 5:
                tt = np.sort(np.repeat(tt[::40], 40)[: len(idx)])
            if h == 1500:
                tt = np.sort(np.repeat(tt[::150], 150)[: len(idx)])
            t[idx] = tt
        ln = rng.choice(np.array([28, 1476, 600], np.uint32), len(host))
        windows.append((host, t, ln, t1))
    st_o, ost = _run_windows(oracle, ctx, bw, 4096, windows, boot=T0 + 30 * MS, ordered=ordered)
    assert (st_o == 1).sum() > 0.9 * len(st_o) * 0.5
    assert (ost["rflags"] & oracle.RL_PENDING).any()  # the slow relays carry tasks over


@pytest.mark.parametrize("ordered,carried", [(False, False), (True, False), (True, True)])
def test_same_time_group_beyond_ring(oracle, ctx, ordered, carried):
    """A same-time group of arrivals larger than the ring: SG_ERR_CAPACITY.  Ordered calls
    too, with and without elements carried from an earlier call in the ring (the
    ordered call's end-of-call id translation must not run over the wrapped ring)."""
    import torch

    bw = np.array([8000 if carried else 10**9, 10**9], np.uint64)  # 1 B/ms: the carried ones stay queued
    ib = InboundPipeline(bw, 16, ctx=ctx)
    st = torch.zeros(64, dtype=torch.uint8, device="cuda")
    fwd = torch.zeros(64, dtype=torch.int64, device="cuda")
    if carried:  # 6 elements queued on host 0 (ids 40..45), one of them cached by the relay
        k = 6
        ib.run(_dev(np.zeros(k), np.uint32, np.int32), _dev(np.full(k, T0), np.uint64, np.int64),
               _dev(np.arange(40, 40 + k), np.uint32, np.int32), _dev(np.full(k, 1500), np.uint32, np.int32),
               T0 + MS, 0, T0 + 10**12, fwd, st)
        assert int(ib.get_state()["tail"][0] - ib.get_state()["head"][0]) >= 4
    host = np.r_[np.zeros(20, np.uint32), np.ones(5, np.uint32)]
    args = (_dev(host, np.uint32, np.int32), _dev(np.full(25, T0 + 2 * MS), np.uint64, np.int64),
            _dev(np.arange(25), np.uint32, np.int32), _dev(np.full(25, 100), np.uint32, np.int32), T0 + 10 * MS,
            0, T0 + 10**12, fwd, st)
    with pytest.raises(ShadowGpuError) as e:
        if ordered:
            ib.run_ordered(*args, torch.zeros(32, dtype=torch.int64, device="cuda"),
                           torch.zeros(32, dtype=torch.uint8, device="cuda"))
        else:
            ib.run(*args)
    assert e.value.code == _capi.SG_ERR_CAPACITY
    torch.cuda.synchronize()  # the device is still usable: no fault


def test_ordered_carried_ids_at_the_top(oracle, ctx):
    """Packets carried from an earlier call with the largest ids allowed (just below 2^31 =
    n_packets): an ordered call writes their fates by packet id and its own arrivals'
    by arrival index (it tells them apart by bit 31, which no packet id may set).  The status and
    forward-time arrays span 2^31 ids (2 GB + 16 GB on the device); the oracle runs the same events
    with the carried ids renumbered 100 + k."""
    import torch

    NB = 64
    BIG = 2**31 - NB  # carried ids BIG + k, the last NB ids below 2^31
    rng = np.random.default_rng(77)
    H = 16
    bw = np.where(np.arange(H) < 8, 8000 * 30, 10**9).astype(np.uint64)  # 30 B/ms on hosts 0-7
    ib = InboundPipeline(bw, 64, ctx=ctx)
    ost = oracle.inbound_state(bw, ib.cap)
    n_all = 2**31
    st_g = torch.zeros(n_all, dtype=torch.uint8, device="cuda")
    fwd_g = torch.full((n_all,), -1, dtype=torch.int64, device="cuda")
    st_o = np.zeros(100 + NB, np.uint8)
    fwd_o = np.full(100 + NB, np.uint64(2**64 - 1))
    ctr_g = torch.zeros(H, dtype=torch.int64, device="cuda")
    ctr_o = np.zeros(H, np.uint64)
    sim_end = T0 + 10**12
    # call 1 (by id): NB arrivals with ids 2^31 + k at one instant, 8 on each slow relay, which
    # forwards one, caches one and leaves six queued
    h1 = np.repeat(np.arange(8), NB // 8).astype(np.uint32)
    t1 = np.full(NB, T0 + MS, np.uint64)
    l1 = np.full(NB, 1500, np.uint32)
    ib.run(_dev(h1, np.uint32, np.int32), _dev(t1, np.uint64, np.int64),
           _dev((BIG + np.arange(NB)).astype(np.uint32), np.uint32, np.int32), _dev(l1, np.uint32, np.int32),
           T0 + 2 * MS, 0, sim_end, fwd_g, st_g, ctr_g.data_ptr())
    oracle.inbound_run(ost, h1, t1, 100 + np.arange(NB, dtype=np.uint32), l1, T0 + 2 * MS, 0, sim_end, ctr_o,
                       fwd_o, st_o)
    got = ib.get_state()
    q = got["tail"] - got["head"]
    assert q.sum() >= 40  # carried elements
    assert (got["ring_pkt"][got["ring_pkt"] != 0] >= BIG).any()
    # call 2 (ordered): 60 arrivals with ids 0..59 over 300 ms; the carried ids leave in it
    n2 = 60
    h2 = np.sort(rng.integers(0, H, n2)).astype(np.uint32)
    t2 = np.sort(rng.integers(T0 + 3 * MS, T0 + 300 * MS, n2)).astype(np.uint64)
    o = np.lexsort((t2, h2))
    h2, t2 = h2[o], t2[o]
    l2 = rng.choice(np.array([28, 1476], np.uint32), n2)
    p2 = np.arange(n2, dtype=np.uint32)
    _run(ib, True, h2, t2, p2, l2, T0 + 400 * MS, 0, sim_end, fwd_g, st_g, ctr_g.data_ptr())
    oracle.inbound_run(ost, h2, t2, p2, l2, T0 + 400 * MS, 0, sim_end, ctr_o, fwd_o, st_o)
    # the carried ids' fates at 2^31 + k, the arrivals' at their ids; nothing else written
    gst = np.r_[st_g[:n2].cpu().numpy(), st_g[BIG:BIG + NB].cpu().numpy()]
    ost_ = np.r_[st_o[:n2], st_o[100:100 + NB]]
    assert np.array_equal(gst, ost_)
    assert (ost_[n2:] == 1).sum() > 40 and (ost_[n2:] == 2).sum() > 8  # carried ids forwarded and dropped
    assert (ost_[:n2] == 0).sum() > 0  # and some of this call's arrivals stay queued (ids translated back)
    assert int(st_g.count_nonzero()) == int((ost_ != 0).sum())
    gfw = np.r_[fwd_g[:n2].cpu().numpy(), fwd_g[BIG:BIG + NB].cpu().numpy()].view(np.uint64)
    ofw = np.r_[fwd_o[:n2], fwd_o[100:100 + NB]]
    assert np.array_equal(gfw[ost_ == 1], ofw[ost_ == 1])
    assert np.array_equal(ctr_g.cpu().numpy().view(np.uint64), ctr_o)
    got = ib.get_state()
    for k in QKEYS + RKEYS:
        assert np.array_equal(got[k], ost[k]), k
    del st_g, fwd_g
    torch.cuda.empty_cache()


@pytest.mark.parametrize("ordered", [False, True])
def test_packet_ids_bounded(ctx, ordered):
    """Packet ids stay below n_packets <= 2^31 (an ordered call marks its arrival indices with
    bit 31): n_packets above 2^31 is refused before any work, and an id at or past n_packets is
    refused as soon as it enters a queue (by id) or would be left queued by an ordered call."""
    import torch

    ib = InboundPipeline(np.array([8000, 10**9], np.uint64), 16, ctx=ctx)  # host 0: 1 B/ms (keeps packets)
    small = torch.zeros(8, dtype=torch.int64, device="cuda")
    huge = torch.zeros(2**31 + 1, dtype=torch.uint8, device="cuda")
    arr = (_dev([0, 0, 0], np.uint32, np.int32), _dev([T0 + MS] * 3, np.uint64, np.int64),
           _dev([0, 1, 2], np.uint32, np.int32), _dev([1500] * 3, np.uint32, np.int32), T0 + 2 * MS, 0, T0 + 10**12)
    with pytest.raises(ShadowGpuError) as e:  # n_packets = 2^31 + 1
        if ordered:
            ib.run_ordered(*arr, small, huge, small, torch.zeros(8, dtype=torch.uint8, device="cuda"))
        else:
            ib.run(*arr, small, huge)
    assert e.value.code == _capi.SG_ERR_INVALID_ARG
    del huge
    torch.cuda.empty_cache()
    st = torch.zeros(4, dtype=torch.uint8, device="cuda")
    fwd = torch.zeros(4, dtype=torch.int64, device="cuda")
    # ids 0, 1 and 7 (>= n_packets = 4): the first is forwarded, the second cached, the third queued
    bad = (arr[0], arr[1], _dev([0, 1, 7], np.uint32, np.int32), *arr[3:])
    with pytest.raises(ShadowGpuError) as e:
        if ordered:
            ib.run_ordered(*bad, fwd, st, small, torch.zeros(8, dtype=torch.uint8, device="cuda"))
        else:
            ib.run(*bad, fwd, st)
    assert e.value.code == _capi.SG_ERR_INVALID_ARG
    torch.cuda.synchronize()
