"""GPU parity of the routers' inbound CoDel queues (sg_codel_*) against the
oracle (router/codel_queue.rs restated; the oracle itself is pinned by the
reference's unit tests in tests/test_codel_cpu.py).  Bit-exact: pop results,
packet statuses and the whole per-host state, across consecutive calls."""
import numpy as np
import pytest

from shadow_amd import ShadowGpuError, _capi
from shadow_amd.router import CoDelEvents, CoDelQueues

pytestmark = pytest.mark.gpu
T0 = 946684800 * 10**9
MS = 10**6
KEYS = ("flags", "interval_end", "drop_next", "cur", "prev", "bytes", "head", "tail")


def _status(n):
    import torch

    return torch.zeros(max(n, 1), dtype=torch.uint8, device="cuda")


def _same_state(O, got, want):
    for k in KEYS:
        assert np.array_equal(got[k], want[k]), k
    # live ring slots only: [head, tail) per host
    cap = want["cap"]
    lo = want["head"].astype(np.int64)
    n = want["tail"].astype(np.int64) - lo
    hh = np.repeat(np.arange(len(n)), n)
    c = lo[hh] + np.arange(int(n.sum())) - np.repeat(np.cumsum(n) - n, n)
    i = hh * cap + (c % cap)
    for k in ("ring_pkt", "ring_ts", "ring_len"):
        assert np.array_equal(got[k][i], want[k][i]), k


def _run_both(O, q, ostate, gstat, ostat, host, kind, t, pkt, ln):
    ev = CoDelEvents.from_numpy(host, kind, t, pkt, ln)
    res, nd = q.run(ev, gstat)
    before = (ostat == 2).sum()
    want = O.codel_run(ostate, host, kind, t, pkt, ln, ostat)
    assert np.array_equal(res.cpu().numpy().view(np.uint32), want)
    assert np.array_equal(gstat.cpu().numpy()[: len(ostat)], ostat)
    assert nd == (ostat == 2).sum() - before
    return want


def _host_times(host, gaps, t0):
    """Per host (host sorted): t0 + the running sum of its own gaps (a segmented cumsum)."""
    c = np.cumsum(gaps.astype(np.int64))
    first = np.r_[True, host[1:] != host[:-1]]
    base = np.maximum.accumulate(np.where(first, c - gaps, 0))
    return (t0 + c - base).astype(np.uint64)


def _stream(rng, H, E, t0, gap_ms, p_pop, n_pkt0=0):
    host = np.sort(rng.integers(0, H, E)).astype(np.uint32)
    kind = (rng.random(E) < p_pop).astype(np.uint8)
    t = _host_times(host, rng.integers(0, gap_ms * MS, E), t0)
    pkt = (n_pkt0 + np.arange(E)).astype(np.uint32)
    ln = rng.integers(40, 1500, E).astype(np.uint32)
    return host, kind, t, pkt, ln


def test_reference_drop_many_sequence(oracle, ctx):
    """codel_queue.rs:494-534 event by event: state equal after every event."""
    q = CoDelQueues(1, 64, ctx=ctx)
    os_ = oracle.codel_state(1, q.cap)
    gstat, ostat = _status(64), np.zeros(64, np.uint8)
    start, end = T0 + 1000 * MS, T0 + 1000000 * MS
    seq = [(0, start)] * 20 + [(1, start + 10 * MS), (1, start + 110 * MS), (1, end)]
    for i, (k, t) in enumerate(seq):
        _run_both(oracle, q, os_, gstat, ostat, [0], [k], [t], [i], [1028])
        _same_state(oracle, q.get_state(), os_)
    st = q.get_state()
    assert st["tail"][0] - st["head"][0] == 1 and st["cur"][0] == 16 and not st["flags"][0] & 1


@pytest.mark.parametrize("gap_ms,p_pop,layout", [(3, 0.45, ""), (1, 0.3, ""), (20, 0.5, ""), (3, 0.45, "0"),
                                                  (1, 0.3, "1")])
def test_random_streams_over_calls(oracle, ctx, monkeypatch, gap_ms, p_pop, layout):
    """500 hosts, three consecutive calls of 60k events: state carries over.  ~120 events
    per host: the blocks take lane-major chunks by default (sg_codel.hip ChunkMap); layout
    forces contiguous ("0") or lane-major ("1") chunks."""
    if layout:
        monkeypatch.setenv("SG_LANE_MAJOR", layout)
    rng = np.random.default_rng(gap_ms)
    H, E = 500, 60000
    q = CoDelQueues(H, 4096, ctx=ctx)
    os_ = oracle.codel_state(H, q.cap)
    gstat, ostat = _status(3 * E), np.zeros(3 * E, np.uint8)
    t0 = T0 + 10**9
    for c in range(3):
        ev = _stream(rng, H, E, t0, gap_ms, p_pop, n_pkt0=c * E)
        _run_both(oracle, q, os_, gstat, ostat, *ev)
        t0 = int(ev[2].max()) + 1
    _same_state(oracle, q.get_state(), os_)
    assert (ostat == 2).any() and (ostat == 1).any()


@pytest.mark.parametrize("layout", ["", "1"])
def test_queue_deeper_than_a_chunk(oracle, ctx, monkeypatch, layout):
    """One host's queue grows past a staged chunk (1024 events) and drains in later
    chunks: its elements are read back from the ring in HBM, which the kernel
    writes only for what outlives each chunk.  Then push/pop cycles wrap the ring
    indices several times.  Neighbour hosts have a few events each.  layout "1":
    lane-major chunks of 16 events per host (the default keeps this block contiguous)."""
    if layout:
        monkeypatch.setenv("SG_LANE_MAJOR", layout)
    rng = np.random.default_rng(5)
    cap = 4096
    q = CoDelQueues(3, cap, ctx=ctx)
    os_ = oracle.codel_state(3, q.cap)
    n_pkt = 40000
    gstat, ostat = _status(n_pkt), np.zeros(n_pkt, np.uint8)
    t0 = T0 + 10**9
    # host 1: 2500 pushes 1 us apart, then 2500 pops 2 ms apart (drop mode), in one call
    h1_kind = np.r_[np.zeros(2500, np.uint8), np.ones(2500, np.uint8)]
    h1_t = np.r_[t0 + np.arange(2500) * 1000, t0 + 3 * MS + np.arange(2500) * 2 * MS].astype(np.uint64)
    host = np.r_[np.zeros(3, np.uint32), np.ones(5000, np.uint32), np.full(3, 2, np.uint32)]
    kind = np.r_[np.array([0, 1, 1], np.uint8), h1_kind, np.array([0, 0, 1], np.uint8)]
    t = np.r_[t0 + np.arange(3) * MS, h1_t, t0 + np.arange(3) * MS].astype(np.uint64)
    pkt = np.arange(len(host), dtype=np.uint32)
    ln = rng.integers(40, 1500, len(host)).astype(np.uint32)
    _run_both(oracle, q, os_, gstat, ostat, host, kind, t, pkt, ln)
    _same_state(oracle, q.get_state(), os_)
    # wrap: calls of bursts (push 600, pop 400) on host 1, queue depth stepping up and down
    tn, p0 = int(t.max()) + MS, len(host)
    for c in range(12):
        k = np.r_[np.zeros(600, np.uint8), np.ones(400 if c % 3 else 900, np.uint8)]
        tt = (tn + np.arange(len(k)) * 50_000).astype(np.uint64)
        hh = np.ones(len(k), np.uint32)
        pp = (p0 + np.arange(len(k))).astype(np.uint32)
        _run_both(oracle, q, os_, gstat, ostat, hh, k, tt, pp, rng.integers(40, 1500, len(k)).astype(np.uint32))
        tn, p0 = int(tt.max()) + MS, p0 + len(k)
    _same_state(oracle, q.get_state(), os_)
    st = q.get_state()
    assert int(st["tail"][1]) > 2 * cap  # the ring indices wrapped
    assert (ostat == 2).any() and (ostat == 1).any()


@pytest.mark.parametrize("layout", ["", "1"])
def test_large_single_call(oracle, ctx, monkeypatch, layout):
    """100k hosts, 1M events (the bench shape), one call; layout "1" forces lane-major chunks."""
    if layout:
        monkeypatch.setenv("SG_LANE_MAJOR", layout)
    rng = np.random.default_rng(11)
    H, E = 100000, 1000000
    q = CoDelQueues(H, 256, ctx=ctx)
    os_ = oracle.codel_state(H, q.cap)
    gstat, ostat = _status(E), np.zeros(E, np.uint8)
    _run_both(oracle, q, os_, gstat, ostat, *_stream(rng, H, E, T0 + 10**9, 30, 0.4))
    _same_state(oracle, q.get_state(), os_)


def test_many_events_per_host(oracle, ctx):
    """The C5 shape per block (~200 events per host, 1 ms round): 6,400 hosts, 1.28M events,
    two calls; the blocks take lane-major chunks."""
    rng = np.random.default_rng(12)
    H, E = 6400, 1280000
    q = CoDelQueues(H, 1024, ctx=ctx)
    os_ = oracle.codel_state(H, q.cap)
    gstat, ostat = _status(2 * E), np.zeros(2 * E, np.uint8)
    t0 = T0 + 10**9
    for c in range(2):
        ev = _stream(rng, H, E, t0, 0.01, 0.5, n_pkt0=c * E)
        _run_both(oracle, q, os_, gstat, ostat, *ev)
        t0 = int(ev[2].max()) + 1
    _same_state(oracle, q.get_state(), os_)


def test_state_roundtrip_and_empty_call(ctx):
    q = CoDelQueues(3, 8, ctx=ctx)
    st = q.get_state()
    st["flags"][1] = 1
    st["bytes"][2] = 77
    q.set_state(st)
    st2 = q.get_state()
    assert st2["flags"][1] == 1 and st2["bytes"][2] == 77
    res, nd = q.run(CoDelEvents.from_numpy([], [], [], [], []), _status(1))
    assert len(res) == 0 and nd == 0


def test_errors(ctx):
    q = CoDelQueues(4, 2, ctx=ctx)  # ring of 2
    with pytest.raises(ShadowGpuError) as e:
        q.run(CoDelEvents.from_numpy([0, 0, 0], [0, 0, 0], [T0] * 3, [0, 1, 2], [100] * 3), _status(8))
    assert e.value.code == _capi.SG_ERR_CAPACITY
    q = CoDelQueues(4, 8, ctx=ctx)
    with pytest.raises(ShadowGpuError) as e:
        q.run(CoDelEvents.from_numpy([2, 1], [0, 0], [T0] * 2, [0, 1], [100] * 2), _status(8))
    assert e.value.code == _capi.SG_ERR_UNSORTED
    with pytest.raises(ShadowGpuError) as e:
        q.run(CoDelEvents.from_numpy([0, 9], [0, 0], [T0] * 2, [0, 1], [100] * 2), _status(8))
    assert e.value.code == _capi.SG_ERR_INVALID_ARG


def test_good_state_mix(oracle, ctx):
    """Most hosts in CoDel's good state (microsecond gaps), a few with queues that
    stand past TARGET and enter drop mode, in the same blocks and chunks; four
    calls, so elements pushed in one call are popped from the ring in the next,
    and hosts cross chunk boundaries."""
    rng = np.random.default_rng(23)
    H, E = 20000, 200000
    q = CoDelQueues(H, 512, ctx=ctx)
    os_ = oracle.codel_state(H, q.cap)
    gstat, ostat = _status(4 * E), np.zeros(4 * E, np.uint8)
    t0 = T0 + 10**9
    slow = rng.random(H) < 0.02
    for c in range(4):
        host = np.sort(rng.integers(0, H, E)).astype(np.uint32)
        # a few hosts get long runs (several chunks' worth of events)
        host[: 3000] = 7
        host[3000: 5500] = 1000 + c
        host = np.sort(host)
        kind = (rng.random(E) < np.where(slow[host], 0.3, 0.5)).astype(np.uint8)
        t = _host_times(host, rng.integers(0, np.where(slow[host], 4 * MS, 2000)), t0)
        pkt = (c * E + np.arange(E)).astype(np.uint32)
        ln = rng.integers(40, 1500, E).astype(np.uint32)
        _run_both(oracle, q, os_, gstat, ostat, host, kind, t, pkt, ln)
        t0 = int(t.max()) + 1
    _same_state(oracle, q.get_state(), os_)
    assert (ostat == 2).any() and (ostat == 1).any()


def test_bytes_below_ring_contents(oracle, ctx):
    """A state whose byte count is below what its ring holds (set_state): pops
    saturate the count at zero (codel_queue.rs pop_front)."""
    H = 64
    q = CoDelQueues(H, 16, ctx=ctx)
    os_ = oracle.codel_state(H, q.cap)
    gstat, ostat = _status(1000), np.zeros(1000, np.uint8)
    t0 = T0 + 10**9
    host = np.repeat(np.arange(H, dtype=np.uint32), 4)
    kind = np.tile(np.array([0, 0, 0, 0], np.uint8), H)
    t = (t0 + np.tile(np.arange(4), H) * 1000).astype(np.uint64)
    pkt = np.arange(4 * H, dtype=np.uint32)
    ln = np.full(4 * H, 1000, np.uint32)
    _run_both(oracle, q, os_, gstat, ostat, host, kind, t, pkt, ln)
    st = q.get_state()
    st["bytes"][::2] = 1500  # below the 4000 queued
    q.set_state(st)
    os_["bytes"][:] = st["bytes"]
    host = np.repeat(np.arange(H, dtype=np.uint32), 3)
    kind = np.ones(3 * H, np.uint8)
    t = (t0 + 10**6 + np.tile(np.arange(3), H) * 1000).astype(np.uint64)
    _run_both(oracle, q, os_, gstat, ostat, host, kind, t, np.zeros(3 * H, np.uint32), np.zeros(3 * H, np.uint32))
    _same_state(oracle, q.get_state(), os_)
