"""The outbound-pipeline oracle (interface fifo -> relay_inet_out token bucket ->
router -> Worker::send_packet) on hand-checkable cases: relay/mod.rs:111-275 (the
forwarding loop, is_local, bootstrapping), relay/mod.rs:278-319 (the bucket's
refill and burst), host.rs:930-945 (notify), router/mod.rs:41-43 (send)."""
import numpy as np
import pytest

T0 = 946684800 * 10**9
MS = 10**6
NEVER = 2**63


def run(O, st, sends, window_end, boot=0, sim_end=NEVER, n_pk=16):
    host, t, pkt, ln, pay, dst = (list(x) for x in zip(*sends)) if sends else ([],) * 6
    ctr = np.zeros(len(st["head"]), np.uint64)
    fwd = np.full(n_pk, np.uint64(2**64 - 1))
    status = np.zeros(n_pk, np.uint8)
    out = O.outbound_run(st, host, t, pkt, ln, pay, dst, window_end, boot, sim_end, ctr, fwd, status)
    return out, ctr, fwd, status


def test_unthrottled_sends_at_notify_time(oracle):
    """1 Gbit/s: every packet leaves at its send time; each send finds the relay Idle
    and schedules one zero-delay forward task (one event id each)."""
    st = oracle.outbound_state([10], [10**9], 8)
    sends = [(0, T0 + 5, 0, 1500, 1460, 99), (0, T0 + 9, 1, 1500, 1460, 98), (0, T0 + 9, 2, 60, 20, 97)]
    out, ctr, fwd, status = run(oracle, st, sends, T0 + MS)
    assert list(out["packet"]) == [0, 1, 2] and list(out["send_time"] - T0) == [5, 9, 9]
    assert list(out["dst_ipv4"]) == [99, 98, 97] and list(out["payload_len"]) == [1460, 1460, 20]
    assert ctr[0] == 2  # the two sends at T0+9 share one task
    assert list(status[:3]) == [1, 1, 1]


def test_bucket_blocks_then_refills(oracle):
    """8 Mbit/s: refill 1000 B per ms, capacity 2500 B.  The second 1500-B packet waits
    for the next refill (RelayCached); the wait is one more event id."""
    st = oracle.outbound_state([10], [8 * 10**6], 8)
    sends = [(0, T0 + 1, 0, 1500, 1472, 11), (0, T0 + 1, 1, 1500, 1472, 11), (0, T0 + 2, 2, 1500, 1472, 11)]
    out, ctr, fwd, status = run(oracle, st, sends, T0 + 10 * MS)
    assert list(out["send_time"] - T0) == [1, MS, 2 * MS]
    assert ctr[0] == 3
    assert st["rflags"][0] == 0 and st["head"][0] == st["tail"][0] == 3


def test_pending_task_carries_over(oracle):
    """A task at or after window_end stays pending; the next window runs it."""
    st = oracle.outbound_state([10], [8 * 10**6], 8)
    sends = [(0, T0 + 1, 0, 1500, 1472, 11), (0, T0 + 1, 1, 1500, 1472, 11)]
    out, ctr, _, status = run(oracle, st, sends, T0 + MS)
    assert list(out["packet"]) == [0] and status[1] == 0
    assert st["rflags"][0] == oracle.RL_PENDING | oracle.RL_CACHED and st["task_time"][0] == T0 + MS
    out2, ctr2, fwd2, status2 = run(oracle, st, [], T0 + 2 * MS)
    assert list(out2["packet"]) == [1] and list(out2["send_time"]) == [T0 + MS] and ctr2[0] == 0


def test_local_packets_skip_the_bucket(oracle):
    """dst == own address: back to the interface without tokens, never to the router
    (relay/mod.rs:222-226, :259-264) -- but in FIFO order behind a blocked packet."""
    st = oracle.outbound_state([10], [8000], 8)  # 1 B per ms: the second packet blocks
    sends = [(0, T0 + 1, 0, 1500, 1472, 11), (0, T0 + 1, 1, 1500, 1472, 10), (0, T0 + 1, 2, 1500, 1472, 11),
             (0, T0 + 1, 3, 40, 0, 10)]
    out, ctr, fwd, status = run(oracle, st, sends, T0 + MS)
    # bucket 1501 B: pkt 0 uses 1500; pkt 1 is local; pkt 2 blocks; pkt 3 waits behind it
    assert list(out["packet"]) == [0] and list(status[:4]) == [1, 2, 0, 0] and fwd[1] == T0 + 1


def test_bootstrapping_has_no_rate_limit(oracle):
    st = oracle.outbound_state([10], [8000], 8)
    sends = [(0, T0 + k, k, 1500, 1472, 11) for k in range(5)]
    out, _, _, _ = run(oracle, st, sends, T0 + MS, boot=T0 + 3)
    # times 0..2 are before bootstrap_end (no limit); the bucket (1501 B) then pays for one more
    assert list(out["packet"]) == [0, 1, 2, 3]


def test_task_past_sim_end_never_runs(oracle):
    st = oracle.outbound_state([10], [8000], 8)
    sends = [(0, T0, 0, 1500, 1472, 11), (0, T0, 1, 1500, 1472, 11)]
    out, _, _, status = run(oracle, st, sends, T0 + 10 * 10**9, sim_end=T0 + MS)
    assert list(out["packet"]) == [0] and status[1] == 0
    assert st["rflags"][0] & oracle.RL_NEVER


def test_errors(oracle):
    st = oracle.outbound_state([10], [10**9], 2)
    with pytest.raises(ValueError, match="-6"):  # a host's times decrease
        run(oracle, st, [(0, T0 + 5, 0, 100, 60, 11), (0, T0 + 4, 1, 100, 60, 11)], T0 + MS)
    st = oracle.outbound_state([10], [8000], 2)
    with pytest.raises(ValueError, match="-2"):  # more than ring_cap queued at once
        run(oracle, st, [(0, T0, k, 1500, 1472, 11) for k in range(3)], T0 + MS)
    st = oracle.outbound_state([10], [10**9], 2)
    with pytest.raises(ValueError, match="-5"):
        run(oracle, st, [(0, T0 + MS, 0, 100, 60, 11)], T0 + MS)
