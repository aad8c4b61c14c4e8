"""The inbound-pipeline oracle (router CoDel -> relay_inet_in token bucket):
its token bucket against the reference's own tests (relay/token_bucket.rs:162-277),
and the relay's forwarding behaviour on hand-checkable cases."""
import numpy as np
import pytest

T0 = 946684800 * 10**9
MS = 10**6


def tb(cap, inc, interval, last):
    return np.array([cap, cap, inc, last, interval], np.uint64)


def test_refill_after_one_interval(oracle):         # token_bucket.rs:189-211
    now = T0 + 1000 * MS
    b = tb(100, 10, 10 * MS, now)
    assert oracle.token_bucket_remove(b, 100, now) == (True, 0)
    for i in range(1, 11):
        ok, bal = oracle.token_bucket_remove(b, 0, now + 10 * MS * i)
        assert ok and bal == 10 * i


def test_refill_after_multiple_intervals(oracle):   # token_bucket.rs:213-228
    now = T0 + 1000 * MS
    b = tb(100, 10, 10 * MS, now)
    assert oracle.token_bucket_remove(b, 100, now)[0]
    assert oracle.token_bucket_remove(b, 0, now + 50 * MS) == (True, 50)


def test_capacity_limit(oracle):                    # token_bucket.rs:230-245
    now = T0 + 1000 * MS
    b = tb(100, 10, 10 * MS, now)
    assert oracle.token_bucket_remove(b, 100, now)[0]
    assert oracle.token_bucket_remove(b, 0, now + 60 * 10**9) == (True, 100)


def test_remove_error(oracle):                      # token_bucket.rs:247-276
    now = T0 + 1000 * MS
    b = tb(100, 10, 125 * MS, now)
    assert oracle.token_bucket_remove(b, 100, now) == (True, 0)
    assert oracle.token_bucket_remove(b, 50, now) == (False, 125 * 5 * MS)
    assert oracle.token_bucket_remove(b, 50, now + 10 * MS) == (False, (125 * 5 - 10) * MS)


def _run(oracle, bw_bits, arrivals, window_end, bootstrap_end=0, sim_end=2**63):
    H = len(bw_bits)
    st = oracle.inbound_state(np.array(bw_bits, np.uint64), 64)
    host, t, pkt, ln = (np.array(x) for x in zip(*arrivals)) if arrivals else ([], [], [], [])
    ctr = np.zeros(H, np.uint64)
    fwd = np.full(64, np.uint64(2**64 - 1))
    status = np.zeros(64, np.uint8)
    oracle.inbound_run(st, host, t, pkt, ln, window_end, bootstrap_end, sim_end, ctr, fwd, status)
    return st, ctr, fwd, status


def test_unthrottled_forwards_at_arrival(oracle):
    """1 Gbit/s down: 125 000 B refill per ms, so each packet is forwarded when it arrives;
    one forward task per arrival (each arrival finds the relay Idle again)."""
    t = T0 + 5 * MS
    st, ctr, fwd, status = _run(oracle, [10**9], [(0, t, 0, 1500), (0, t + 1000, 1, 1500)], T0 + 10 * MS)
    assert list(fwd[:2]) == [t, t + 1000] and list(status[:2]) == [1, 1]
    assert ctr[0] == 2 and st["rflags"][0] == 0


def test_same_time_arrivals_share_one_task(oracle):
    """Packet events before the Local forward task at the same time (event.rs:103-112):
    three arrivals at t, one task at t forwards all three."""
    t = T0 + 5 * MS
    st, ctr, fwd, status = _run(oracle, [10**9], [(0, t, k, 100) for k in range(3)], T0 + 10 * MS)
    assert list(fwd[:3]) == [t] * 3 and ctr[0] == 1


def test_throttled_relay_caches_and_reschedules(oracle):
    """8 kbit/s down = 1 B per 1 ms refill, capacity 1501 B: the second 1500 B packet waits
    1499 refills (token_bucket.rs:93-118), the third stays behind the window end."""
    t = T0 + 5 * MS
    st, ctr, fwd, status = _run(oracle, [8000], [(0, t, k, 1500) for k in range(3)], T0 + 3000 * MS)
    assert fwd[0] == t and status[0] == 1
    # balance 1 after the first; 1499 more tokens are needed: 1499 refills, the first at the next 1 ms boundary
    assert fwd[1] == T0 + 5 * MS + 1499 * MS and status[1] == 1
    assert status[2] == 0 and st["rflags"][0] & oracle.RL_PENDING and st["rflags"][0] & oracle.RL_CACHED
    assert st["task_time"][0] == T0 + 5 * MS + 2999 * MS


def test_bootstrapping_ignores_the_rate_limit(oracle):
    t = T0 + 5 * MS
    st, ctr, fwd, status = _run(oracle, [8000], [(0, t, k, 1500) for k in range(3)], T0 + 10 * MS,
                                bootstrap_end=T0 + 100 * MS)
    assert list(fwd[:3]) == [t] * 3


def test_arrival_past_window_rejected(oracle):
    with pytest.raises(ValueError):
        _run(oracle, [10**9], [(0, T0 + 20 * MS, 0, 100)], T0 + 10 * MS)
