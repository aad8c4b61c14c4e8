"""The outbound-pipeline oracle (interface fifo -> relay_inet_out token bucket ->
router -> Worker::send_packet) on hand-checkable cases: relay/mod.rs:111-275 (the
forwarding loop, is_local, bootstrapping), relay/mod.rs:278-319 (the bucket's
refill and burst), host.rs:930-945 (notify), router/mod.rs:41-43 (send)."""
import numpy as np
import pytest

T0 = 946684800 * 10**9
MS = 10**6
NEVER = 2**63


PACKET = 2**64 - 1  # sends made by a Packet event (event.rs:103-112)


def run(O, st, sends, window_end, boot=0, sim_end=NEVER, n_pk=16, keys=None, ctr0=0):
    """keys: per send (event created at, event id) of the event that made it, or None."""
    host, t, pkt, ln, pay, dst = (list(x) for x in zip(*sends)) if sends else ([],) * 6
    ctr = np.full(len(st["head"]), ctr0, np.uint64)
    fwd = np.full(n_pk, np.uint64(2**64 - 1))
    status = np.zeros(n_pk, np.uint8)
    born = eid = None
    if keys is not None:
        born = np.array([k[0] for k in keys], np.uint64)
        eid = np.array([k[1] for k in keys], np.uint64)
    out = O.outbound_run(st, host, t, pkt, ln, pay, dst, window_end, boot, sim_end, ctr, fwd, status,
                         event_id=eid, event_created=born)
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


# ---- same-time order of a send and a forward task (event.rs:84-155, relay/mod.rs:145-157) ----
# 8 Mbit/s: refill 1000 B per ms, capacity 2500.  Send A (T0+1) finds the relay Idle: task X
# (id 100, created T0+1) runs after the sending event (id 5) and forwards A; B blocks (1000 B
# left) and is cached; the wake-up W (id 101) is created at T0+1 for T0+1ms.  Send C lands on
# T0+1ms exactly.  Who runs first at T0+1ms depends on when C's event was created.
AB = [(0, T0 + 1, 0, 1500, 1472, 11), (0, T0 + 1, 1, 1500, 1472, 11)]
C_AT_WAKE = (0, T0 + MS, 2, 1500, 1472, 11)


@pytest.mark.parametrize("c_key,want_ctr", [
    ((T0, 6), 103),              # C's event created before W (T0 < T0+1): C joins W's run (X, W, W2)
    ((PACKET, PACKET), 103),     # a Packet event's send precedes every Local event
    ((T0 + MS // 2, 7), 104),    # created after W (a timer set at T0+0.5ms): W first (X, W, X2, W2)
    ((T0 + 1, 50), 103),         # same creation time, smaller id: created before W
    ((T0 + 1, 150), 153),        # same creation time, larger id: after W; X2 and W2 numbered past 150
])
def test_wake_vs_send_at_the_same_time(oracle, c_key, want_ctr):
    st = oracle.outbound_state([10], [8 * 10**6], 8)
    keys = [(T0, 5), (T0, 5), c_key]
    out, ctr, fwd, status = run(oracle, st, AB + [C_AT_WAKE], T0 + 10 * MS, keys=keys, ctr0=100)
    assert list(out["packet"]) == [0, 1, 2]
    # B leaves with W at T0+1ms either way; C waits for the next refill either way
    assert list(out["send_time"] - T0) == [1, MS, 2 * MS]
    assert ctr[0] == want_ctr and st["task_id"][0] == want_ctr - 1
    assert st["task_time"][0] == T0 + 2 * MS and st["task_born"][0] == T0 + MS


def test_wake_first_counts_one_more_task(oracle):
    """The two orders differ in the host's event count: the wake-first order empties the
    queue, so C's notify schedules one more task (host.rs:649-653)."""
    got = {}
    for name, ck in (("send_first", (T0, 6)), ("wake_first", (T0 + MS // 2, 7))):
        st = oracle.outbound_state([10], [8 * 10**6], 8)
        _, ctr, _, _ = run(oracle, st, AB + [C_AT_WAKE], T0 + 10 * MS, keys=[(T0, 5), (T0, 5), ck], ctr0=100)
        got[name] = (int(ctr[0]), int(st["task_id"][0]), int(st["task_born"][0]))
    assert got["send_first"] == (103, 102, T0 + MS)  # W2 created by W at T0+1ms
    assert got["wake_first"] == (104, 103, T0 + MS)  # W2 created by X2


def test_notify_task_vs_later_event_at_the_same_time(oracle):
    """X (notify at T0+5 by event 5) and a send at T0+5 by an event created at T0+5 after X
    (id 120 > 100): X runs first and forwards A alone; B's notify finds the relay Idle and
    schedules X2, numbered after B's event (121).  Without keys B joins X's run."""
    sends = [(0, T0 + 5, 0, 100, 60, 11), (0, T0 + 5, 1, 100, 60, 11)]
    st = oracle.outbound_state([10], [10**9], 8)
    out, ctr, _, _ = run(oracle, st, sends, T0 + MS, keys=[(T0, 5), (T0 + 5, 120)], ctr0=100)
    assert list(out["send_time"] - T0) == [5, 5] and ctr[0] == 122 and st["task_id"][0] == 121
    st = oracle.outbound_state([10], [10**9], 8)
    out, ctr, _, _ = run(oracle, st, sends, T0 + MS, ctr0=100)
    assert list(out["send_time"] - T0) == [5, 5] and ctr[0] == 101 and st["task_id"][0] == 100


def test_keys_must_follow_execution_order(oracle):
    st = oracle.outbound_state([10], [10**9], 8)
    sends = [(0, T0 + 5, 0, 100, 60, 11), (0, T0 + 5, 1, 100, 60, 11)]
    with pytest.raises(ValueError, match="-6"):  # a Packet-event send after a Local one, same time
        run(oracle, st, sends, T0 + MS, keys=[(T0, 5), (PACKET, PACKET)])
    st = oracle.outbound_state([10], [10**9], 8)
    with pytest.raises(ValueError, match="-6"):  # Local events out of id order
        run(oracle, st, sends, T0 + MS, keys=[(T0, 9), (T0, 5)])
    st = oracle.outbound_state([10], [10**9], 8)
    run(oracle, st, sends, T0 + MS, keys=[(PACKET, PACKET), (T0, 5)])  # Packet first: fine


def test_tie_task_runs_after_a_later_numbered_event_exists(oracle):
    """A, B, B2 at T0+1 (8 Mbit/s): X (100) forwards A, B blocks, wake-up W (101, created
    T0+1) for T0+1ms.  Send C at T0+1ms by an event created at T0+1 with id 150: W's key
    (T0+1, 101) is smaller, so W runs first -- after event 150 was created.  W forwards B,
    B2 blocks and W reschedules itself: the new wake-up is numbered past 150 (151), not 102
    (the host's counter counts every event created before the task ran, event.rs:84-155)."""
    st = oracle.outbound_state([10], [8 * 10**6], 8)
    sends = AB + [(0, T0 + 1, 3, 1500, 1472, 11), C_AT_WAKE]
    out, ctr, _, status = run(oracle, st, sends, T0 + MS + 1, keys=[(T0, 5)] * 3 + [(T0 + 1, 150)], ctr0=100,
                              n_pk=4)
    assert list(out["packet"]) == [0, 1] and list(status) == [1, 1, 0, 0]
    assert st["task_id"][0] == 151 and st["task_born"][0] == T0 + MS and st["task_time"][0] == T0 + 2 * MS
    assert ctr[0] == 152  # C's notify finds the relay waiting: no new task


def test_send_with_the_pending_tasks_key_is_rejected(oracle):
    """Two events cannot share (created, id): a send made by the key of the pending wake-up
    W (T0+1, 101) at W's time has no execution order and is refused (-6)."""
    st = oracle.outbound_state([10], [8 * 10**6], 8)
    with pytest.raises(ValueError, match="-6"):
        run(oracle, st, AB + [C_AT_WAKE], T0 + 10 * MS, keys=[(T0, 5), (T0, 5), (T0 + 1, 101)], ctr0=100)
    st = oracle.outbound_state([10], [8 * 10**6], 8)  # one id further on: fine
    run(oracle, st, AB + [C_AT_WAKE], T0 + 10 * MS, keys=[(T0, 5), (T0, 5), (T0 + 1, 102)], ctr0=100)
