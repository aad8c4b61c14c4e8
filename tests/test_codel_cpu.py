"""The CoDel oracle (router/codel_queue.rs) against the reference's own unit
tests (codel_queue.rs:332-534, router/mod.rs:81-109), restated through the
batch interface: one host, events fed one at a time so the intermediate queue
length, mode and drop counts can be checked exactly as the reference does."""
import math

import numpy as np

T0 = 946684800 * 10**9             # EmulatedTime::SIMULATION_START
MS = 10**6
MOCK_LEN = 20 + 8 + 1000           # PacketRc::new_ipv4_udp_mock: IPv4 + UDP headers + 1000 B payload


def mock_time_millis(ms):           # network/mod.rs:26-29
    return T0 + ms * MS


class OneQueue:
    def __init__(self, O, cap=64):
        self.O = O
        self.s = O.codel_state(1, cap)
        self.status = np.zeros(256, np.uint8)
        self.next_pkt = 0

    def push(self, now):
        p = self.next_pkt
        self.next_pkt += 1
        self.O.codel_run(self.s, [0], [self.O.CD_PUSH], [now], [p], [MOCK_LEN], self.status)
        return p

    def pop(self, now):
        r = self.O.codel_run(self.s, [0], [self.O.CD_POP], [now], [0], [0], self.status)
        return None if r[0] == self.O.CD_NONE else int(r[0])

    def __len__(self):
        return int(self.s["tail"][0] - self.s["head"][0])

    @property
    def drop_mode(self):
        return bool(self.s["flags"][0] & self.O.CD_DROP)

    @property
    def interval_end(self):
        return int(self.s["interval_end"][0]) if self.s["flags"][0] & self.O.CD_HAS_IEND else None

    @property
    def drop_next(self):
        return int(self.s["drop_next"][0]) if self.s["flags"][0] & self.O.CD_HAS_DNEXT else None


def test_empty(oracle):                       # codel_queue.rs:332-340
    q = OneQueue(oracle)
    assert len(q) == 0 and q.pop(mock_time_millis(1000)) is None


def test_push_pop_simple(oracle):             # codel_queue.rs:342-363, router/mod.rs:89-109
    q = OneQueue(oracle)
    now = mock_time_millis(1000)
    for i in range(1, 11):
        assert len(q) == i - 1
        q.push(now)
        assert len(q) == i
    for i in range(1, 11):
        assert len(q) == 10 - i + 1
        assert q.pop(now) is not None
        assert len(q) == 10 - i
    assert q.pop(now) is None


def test_control_law(oracle):                 # codel_queue.rs:365-386
    now = mock_time_millis(1000)
    interval = oracle.CODEL_INTERVAL_NS
    for i in range(2):
        assert oracle.codel_control_law(now, i) - now == interval
    for i in range(2, 20):
        want = int(math.floor(interval / math.sqrt(i) + 0.5))  # f64::round (no ties here)
        assert oracle.codel_control_law(now, i) - now == want


def test_interval_through_pops(oracle):       # codel_queue.rs:388-431, observed through pop()
    start = mock_time_millis(1000)
    target, interval = oracle.CODEL_TARGET_NS, oracle.CODEL_INTERVAL_NS
    q = OneQueue(oracle)
    for _ in range(5):
        q.push(start)
    assert q.s["bytes"][0] > oracle.CODEL_MTU
    q.pop(start + target - MS)                # below target: no interval
    assert q.interval_end is None
    q.pop(start + target)                     # reached target: interval set, no drop
    assert q.interval_end == start + target + interval and not q.drop_mode
    assert (q.status == 2).sum() == 0


def test_mode(oracle):                        # codel_queue.rs:433-483
    start = mock_time_millis(1000)
    target, interval = oracle.CODEL_TARGET_NS, oracle.CODEL_INTERVAL_NS
    q = OneQueue(oracle)
    for _ in range(6):
        q.push(start)
    assert q.s["bytes"][0] > oracle.CODEL_MTU and len(q) == 6 and not q.drop_mode
    q.pop(start + target - MS)
    assert len(q) == 5 and not q.drop_mode
    q.pop(start + target)
    assert len(q) == 4 and not q.drop_mode
    q.pop(start + target + interval - MS)
    assert len(q) == 3 and not q.drop_mode
    q.pop(start + target + interval)          # enter drop mode, drop one packet
    assert len(q) == 1 and q.drop_mode
    for _ in range(3):
        q.push(start + target + 2 * interval - MS)
    q.pop(start + target + 2 * interval)
    assert not q.drop_mode


def test_drop_empty(oracle):                  # codel_queue.rs:485-492
    q = OneQueue(oracle)
    q.s["flags"][0] |= oracle.CD_DROP
    q.pop(mock_time_millis(1000))
    assert not q.drop_mode


def test_drop_many(oracle):                   # codel_queue.rs:494-534
    start, end = mock_time_millis(1000), mock_time_millis(1000000)
    target, interval = oracle.CODEL_TARGET_NS, oracle.CODEL_INTERVAL_NS
    q = OneQueue(oracle)
    N = 20
    for _ in range(N):
        q.push(start)
    assert len(q) == N and not q.drop_mode
    q.pop(start + target)
    assert len(q) == N - 1 and q.s["cur"][0] == 0 and q.s["prev"][0] == 0 and not q.drop_mode
    q.pop(start + target + interval)
    assert len(q) == N - 3 and q.s["cur"][0] == 1 and q.s["prev"][0] == 1
    assert q.drop_next is not None and q.drop_mode
    assert end >= q.drop_next                 # should_drop(end)
    q.pop(end)
    assert len(q) == 1 and q.s["cur"][0] == N - 4 and not q.drop_mode
    # every packet left exactly once: dequeued (1) or dropped (2); one still queued
    assert (q.status[:N] == 1).sum() + (q.status[:N] == 2).sum() == N - 1


def test_batched_equals_one_at_a_time(oracle):
    """A whole multi-host event stream in one call == the same events one call each."""
    rng = np.random.default_rng(5)
    H, E = 7, 3000
    host = np.sort(rng.integers(0, H, E)).astype(np.uint32)
    kind = (rng.random(E) < 0.45).astype(np.uint8)
    t = np.zeros(E, np.uint64)
    for h in range(H):
        idx = np.nonzero(host == h)[0]
        t[idx] = T0 + np.cumsum(rng.integers(0, 3 * MS, len(idx))).astype(np.uint64)
    pkt = np.arange(E, dtype=np.uint32)
    ln = rng.integers(40, 1500, E).astype(np.uint32)
    s1, st1 = oracle.codel_state(H, 4096), np.zeros(E, np.uint8)
    r1 = oracle.codel_run(s1, host, kind, t, pkt, ln, st1)
    s2, st2 = oracle.codel_state(H, 4096), np.zeros(E, np.uint8)
    r2 = np.array([oracle.codel_run(s2, host[i:i + 1], kind[i:i + 1], t[i:i + 1], pkt[i:i + 1], ln[i:i + 1], st2)[0]
                   for i in range(E)], np.uint32)
    assert np.array_equal(r1, r2) and np.array_equal(st1, st2)
    for k in s1:
        if k != "cap":
            assert np.array_equal(s1[k], s2[k]), k
    assert (st1 == 2).any() and (st1 == 1).any()  # the stream reaches drop mode
