"""The multi-threaded CPU baselines of the lane legs (sgo_{codel,inbound,outbound}_run_mt:
hosts dealt round-robin over threads, as Shadow's worker pool deals them,
thread_per_core.rs:62-64) give exactly the single-thread results: state, statuses,
forward times, event counters and (outbound) the sent packets up to their grouping."""
import numpy as np
import pytest

T0 = 946684800 * 10**9
MS = 10**6


def _grouped(rng, H, n, t0, t1):
    host = np.sort(rng.integers(0, H, n)).astype(np.uint32)
    t = rng.integers(t0, t1, n).astype(np.uint64)
    o = np.lexsort((t, host))
    return host[o], t[o]


def _same_state(a, b):
    for k in a:
        if isinstance(a[k], np.ndarray):
            assert np.array_equal(a[k], b[k]), k


@pytest.mark.parametrize("threads", [2, 5, 16])
def test_codel_mt(oracle, threads):
    rng = np.random.default_rng(threads)
    H, n = 500, 40000
    host, t = _grouped(rng, H, n, T0, T0 + 200 * MS)
    kind = (rng.random(n) < 0.45).astype(np.uint8)
    pkt = np.arange(n, dtype=np.uint32)
    ln = rng.choice(np.array([60, 1500], np.uint32), n)
    out = []
    for th in (1, threads):
        st = oracle.codel_state(H, 1024)
        status = np.zeros(n, np.uint8)
        res = oracle.codel_run(st, host, kind, t, pkt, ln, status, threads=th)
        out.append((st, status, res))
    _same_state(out[0][0], out[1][0])
    assert np.array_equal(out[0][1], out[1][1]) and np.array_equal(out[0][2], out[1][2])
    assert (out[0][1] == 2).any()  # CoDel dropped some


@pytest.mark.parametrize("threads", [3, 16])
def test_inbound_mt(oracle, threads):
    rng = np.random.default_rng(10 + threads)
    H, n = 400, 30000
    bw = rng.integers(10**6, 10**7, H).astype(np.uint64)
    out = []
    for th in (1, threads):
        st = oracle.inbound_state(bw, 4096)
        ctr = np.zeros(H, np.uint64)
        fwd = np.full(2 * n, np.uint64(2**64 - 1))
        status = np.zeros(2 * n, np.uint8)
        r = np.random.default_rng(99)
        for w in range(2):  # two windows: tasks carried over
            host, t = _grouped(r, H, n, T0 + w * 50 * MS, T0 + (w + 1) * 50 * MS)
            ln = r.choice(np.array([28, 1476], np.uint32), n)
            pkt = np.arange(w * n, (w + 1) * n, dtype=np.uint32)
            oracle.inbound_run(st, host, t, pkt, ln, T0 + (w + 1) * 50 * MS, 0, T0 + 10**12, ctr, fwd, status,
                               threads=th)
        out.append((st, ctr, fwd, status))
    _same_state(out[0][0], out[1][0])
    for a, b in zip(out[0][1:], out[1][1:]):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("threads", [4, 16])
def test_outbound_mt(oracle, threads):
    rng = np.random.default_rng(20 + threads)
    H, n = 300, 20000
    ip = (np.arange(H, dtype=np.uint32) + 0x0B000000).astype(np.uint32)
    bw = rng.integers(10**6, 10**8, H).astype(np.uint64)
    host, t = _grouped(rng, H, n, T0, T0 + 30 * MS)
    dst = np.where(rng.random(n) < 0.1, ip[host], ip[rng.integers(0, H, n)]).astype(np.uint32)
    ln = rng.choice(np.array([60, 1500], np.uint32), n)
    pay = (ln - 28).astype(np.uint32)
    pkt = np.arange(n, dtype=np.uint32)
    out = []
    for th in (1, threads):
        st = oracle.outbound_state(ip, bw, 1024)
        ctr = np.zeros(H, np.uint64)
        fwd = np.full(n, np.uint64(2**64 - 1))
        status = np.zeros(n, np.uint8)
        sent = oracle.outbound_run(st, host, t, pkt, ln, pay, dst, T0 + 30 * MS, 0, T0 + 10**12, ctr, fwd, status,
                                   threads=th)
        o = np.argsort(sent["src_host"], kind="stable")
        out.append((st, ctr, fwd, status, {k: v[o] for k, v in sent.items()}))
    _same_state(out[0][0], out[1][0])
    for a, b in zip(out[0][1:4], out[1][1:4]):
        assert np.array_equal(a, b)
    for k in out[0][4]:
        assert np.array_equal(out[0][4][k], out[1][4][k]), k
    assert len(out[0][4]["packet"]) > 0
