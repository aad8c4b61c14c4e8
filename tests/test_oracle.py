"""Pin the CPU oracle (oracle/sg_oracle.c) before trusting it as the GPU checker.

CPU-only.  Anchors: the reference's own unit tests and config (graph/mod.rs,
configuration.rs), the upstream xoshiro256++ vector, scipy's integer Dijkstra,
and an independent pure-Python lexicographic Dijkstra with numpy f32 arithmetic.
"""
import heapq
import json
import os

import numpy as np
import pytest

from shadow_amd import synth

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def kat():
    with open(os.path.join(GOLD, "reference_kat.json")) as f:
        return json.load(f)


# ---- reference known answers --------------------------------------------------
@pytest.mark.parametrize("directed", [True, False])
def test_reference_shortest_path_latencies(oracle, directed):
    """graph/mod.rs:564-651 test_shortest_path (all 9 pairs, both modes)."""
    k = kat()["test_shortest_path"]
    e = np.array(k["edges"])
    rc, lat, loss, _ = oracle.shortest_paths(3, e[:, 0], e[:, 1], e[:, 2], np.zeros(len(e)), directed, [0, 1, 2])
    assert rc == oracle.OK
    want = k["directed_latency" if directed else "undirected_latency"]
    assert lat.tolist() == want
    assert (loss == 0).all()


def test_reference_path_add(oracle):
    """graph/mod.rs:519-533 test_path_add, plus the exact f32 bits of the fold."""
    k = kat()["test_path_add"]
    lat, loss = oracle.path_add(k["a"][0], k["a"][1], k["b"][0], k["b"][1])
    assert lat == k["latency"]
    assert abs(float(loss) - k["loss_approx"]) < k["tol"]
    one = np.float32(1)
    want = one - (one - np.float32(0.35)) * (one - np.float32(0.85))  # numpy f32: one rounding per op
    assert np.float32(loss).view(np.uint32) == np.float32(want).view(np.uint32)
    # the first hop is not the identity: default() + e != e  (graph/mod.rs:322-331)
    _, l1 = oracle.path_add(0, 0.0, 5, 0.1)
    assert np.float32(l1) != np.float32(0.1)


def test_one_gbit_switch(oracle):
    """configuration.rs:1366-1380: single node, self-loop 1 ms, loss 0.0."""
    rc, lat, loss, _ = oracle.shortest_paths(1, [0], [0], [1_000_000], [0.0], False, [0])
    assert rc == oracle.OK and lat.tolist() == [[1_000_000]] and loss.tolist() == [[0.0]]
    rc, lat, loss, _ = oracle.direct_paths(1, [0], [0], [1_000_000], [0.0], False, [0])
    assert rc == oracle.OK and lat.tolist() == [[1_000_000]]


def test_xoshiro_upstream_vector(oracle):
    s = np.array([1, 2, 3, 4], np.uint64)
    assert [oracle.xoshiro_next_u64(s) for _ in range(6)] == kat()["xoshiro256pp_state_1234"]["outputs"]


def test_rng_vectors_frozen(oracle):
    with open(os.path.join(GOLD, "rng_vectors.json")) as f:
        v = json.load(f)
    for seed in (0, 1, 42, 2**63 + 5):
        s = oracle.xoshiro_seed(seed)
        assert [int(x) for x in s] == v[str(seed)]["state"]
        assert [oracle.xoshiro_next_f64(s) for _ in range(8)] == v[str(seed)]["f64"]
    for name, seed in v["host_seed_general1"].items():
        assert oracle.host_seed(1, name) == seed
        assert synth.host_seed(1, name) == seed  # the product-side (Python) derivation agrees


def test_f64_draw_formula(oracle):
    s = oracle.xoshiro_seed(7)
    s2 = s.copy()
    x = oracle.xoshiro_next_u64(s2)
    assert oracle.xoshiro_next_f64(s) == (x >> 11) * 2.0 ** -53


# ---- cross-checks on random graphs --------------------------------------------
def _scipy_latency(g, used):
    import scipy.sparse as sp
    from scipy.sparse.csgraph import dijkstra

    n = g["n"]
    src, dst, lat = g["src"].astype(np.int64), g["dst"].astype(np.int64), g["lat"].astype(np.float64)
    keep = src != dst
    src, dst, lat = src[keep], dst[keep], lat[keep]
    if not g["directed"]:
        src, dst, lat = np.concatenate([src, dst]), np.concatenate([dst, src]), np.concatenate([lat, lat])
    # parallel arcs: keep the minimum
    best = {}
    for s, d, l in zip(src, dst, lat):
        if (s, d) not in best or l < best[(s, d)]:
            best[(s, d)] = l
    r = np.array([k[0] for k in best]); c = np.array([k[1] for k in best]); w = np.array(list(best.values()))
    m = sp.csr_matrix((w, (r, c)), shape=(n, n))
    d = dijkstra(m, directed=True, indices=used)
    return d[:, used]


@pytest.mark.parametrize("directed", [False, True])
def test_oracle_latency_matches_scipy(oracle, directed):
    g = synth.ring_chords_graph(300, 5.0, seed=21, directed=directed, parallel=0.2)
    used = np.random.default_rng(0).permutation(300)[:120].astype(np.uint32)
    rc, lat, _, _ = oracle.shortest_paths(g["n"], g["src"], g["dst"], g["lat"], g["loss"], directed, used, threads=4)
    assert rc == 0
    ref = _scipy_latency(g, used)
    off = ~np.eye(len(used), dtype=bool)
    assert np.array_equal(lat[off].astype(np.float64), ref[off])  # integer ns < 2^53: exact in f64


def _py_lex_dijkstra(g, src):
    """Independent lexicographic Dijkstra over (int latency, numpy f32 loss) with the left fold."""
    n = g["n"]
    adj = [[] for _ in range(n)]
    for s, d, l, p in zip(g["src"], g["dst"], g["lat"], g["loss"]):
        adj[s].append((d, int(l), np.float32(p)))
        if not g["directed"] and s != d:
            adj[d].append((s, int(l), np.float32(p)))
    one = np.float32(1)
    best = {src: (0, np.float32(0))}
    heap = [(0, 0.0, src)]
    done = set()
    while heap:
        l, p, u = heapq.heappop(heap)
        if u in done:
            continue
        done.add(u)
        bl, bp = best[u]
        for v, el, ep in adj[u]:
            if v in done:
                continue
            cand = (bl + el, np.float32(one - np.float32(np.float32(one - bp) * np.float32(one - ep))))
            if v not in best or (cand[0], float(cand[1])) < (best[v][0], float(best[v][1])):
                best[v] = cand
                heapq.heappush(heap, (cand[0], float(cand[1]), v))
    return best


def test_oracle_loss_bits_match_independent_dijkstra(oracle):
    g = synth.ring_chords_graph(60, 5.0, seed=31, parallel=0.3)
    g["loss"] = np.random.default_rng(2).uniform(0, 0.3, len(g["src"])).astype(np.float32)
    g["lat"] = (np.random.default_rng(3).integers(1, 6, len(g["src"])) * 1000).astype(np.uint64)  # many ties
    used = np.arange(60, dtype=np.uint32)
    rc, lat, loss, _ = oracle.shortest_paths(60, g["src"], g["dst"], g["lat"], g["loss"], False, used)
    assert rc == 0
    for s in range(0, 60, 7):
        best = _py_lex_dijkstra(g, s)
        for v in range(60):
            if v == s:
                continue
            assert lat[s, v] == best[v][0]
            assert loss[s, v].view(np.uint32) == np.float32(best[v][1]).view(np.uint32), (s, v)


def test_left_fold_differs_from_tree_fold():
    """Why Floyd-Warshall cannot be used for loss: association changes f32 bits."""
    one = np.float32(1)
    f = lambda a, b: np.float32(one - np.float32(np.float32(one - a) * np.float32(one - b)))
    rng = np.random.default_rng(0)
    diff = 0
    for _ in range(2000):
        e = rng.uniform(0, 0.5, 4).astype(np.float32)
        left = f(f(f(f(np.float32(0), e[0]), e[1]), e[2]), e[3])
        tree = f(f(f(np.float32(0), e[0]), e[1]), f(e[2], e[3]))
        diff += left != tree
    assert diff > 0


# ---- error behaviour ------------------------------------------------------------
def test_errors(oracle):
    # missing self-loop on node 1 (graph/mod.rs:266-268)
    rc, *_ , pair = oracle.shortest_paths(2, [0, 0], [0, 1], [5, 5], [0, 0], False, [0, 1])
    assert rc == oracle.ERR_NO_EDGE and pair == (1, 1)
    # two self-loops on node 0 (graph/mod.rs:269-275)
    rc, *_ , pair = oracle.shortest_paths(2, [0, 0, 1, 0], [0, 0, 1, 1], [5, 6, 5, 5], [0] * 4, False, [0, 1])
    assert rc == oracle.ERR_MULTI_EDGE and pair == (0, 0)
    # unreachable (graph/mod.rs:219 panics): directed 0 -> 1 only
    rc, *_ , pair = oracle.shortest_paths(2, [0, 1, 0], [0, 1, 1], [5, 5, 5], [0] * 3, True, [0, 1])
    assert rc == oracle.ERR_UNREACHABLE and pair == (1, 0)
    # an unused isolated node is fine
    rc, *_ = oracle.shortest_paths(3, [0, 1, 0, 2], [0, 1, 1, 2], [5, 5, 5, 5], [0] * 4, False, [0, 1])
    assert rc == oracle.OK
    # direct paths: missing pair / duplicate pair (undirected counts both stored directions)
    rc, *_ , pair = oracle.direct_paths(2, [0, 1], [0, 1], [5, 5], [0, 0], False, [0, 1])
    assert rc == oracle.ERR_NO_EDGE and pair == (0, 1)
    rc, *_ , pair = oracle.direct_paths(2, [0, 1, 0, 1], [0, 1, 1, 0], [5, 5, 5, 7], [0] * 4, False, [0, 1])
    assert rc == oracle.ERR_MULTI_EDGE and pair == (0, 1)
    rc, lat, *_ = oracle.direct_paths(2, [0, 1, 0, 1], [0, 1, 1, 0], [5, 5, 5, 7], [0] * 4, True, [0, 1])
    assert rc == oracle.OK and lat.tolist() == [[5, 5], [7, 5]]


def test_golden_routing_frozen(oracle):
    z = np.load(os.path.join(GOLD, "routing_small.npz"))
    names = sorted({k.split(".")[0] for k in z.files})
    for name in names:
        g = {k: z[f"{name}.{k}"] for k in ("src", "dst", "lat", "loss")}
        rc, lat, loss, _ = oracle.shortest_paths(int(z[f"{name}.n"][0]), g["src"], g["dst"], g["lat"], g["loss"],
                                                 bool(z[f"{name}.directed"][0]), z[f"{name}.used"], threads=4)
        assert rc == 0
        assert np.array_equal(lat, z[f"{name}.out_lat"]), name
        assert np.array_equal(loss.view(np.uint32), z[f"{name}.out_loss"].view(np.uint32)), name


# ---- delivery semantics ---------------------------------------------------------
def _tiny_world():
    lat = np.array([[1000, 5000], [5000, 2000]], np.uint64)
    loss = np.array([[0.0, 0.5], [0.5, 0.0]], np.float32)
    host_ip = np.array([100, 200], np.uint32)
    host_row = np.array([0, 1], np.uint32)
    return lat, loss, host_ip, host_row


def test_deliver_semantics(oracle):
    lat, loss, host_ip, host_row = _tiny_world()
    rng = np.stack([oracle.xoshiro_seed(9), oracle.xoshiro_seed(10)])
    ctr = np.array([5, 0], np.uint64)
    # host 0 sends: after-sim-end, unknown dst, ack (payload 0) x3, data x3
    src = [0] * 8
    dst = [200, 999, 200, 200, 200, 200, 200, 200]
    pay = [10, 10, 0, 0, 0, 10, 10, 10]
    t = [10_000, 100, 100, 200, 300, 400, 500, 600]
    sim_end = 10_000
    r = oracle.deliver_round(1000, sim_end, 0, src, dst, pay, t, host_ip, host_row, lat, loss, rng, ctr)
    st = r["status"].tolist()
    assert st[0] == oracle.ST_SIM_END and st[1] == oracle.ST_DROP_NO_DST
    assert st[2:5] == [oracle.ST_DELIVERED] * 3  # acks are never dropped (worker.rs:362-368)
    # draws: exactly one per resolved packet, in send order
    s = oracle.xoshiro_seed(9)
    draws = [oracle.xoshiro_next_f64(s) for _ in range(6)]
    rel = float(np.float32(1) - np.float32(0.5))
    for k in range(3):
        want = oracle.ST_DROP_LOSS if draws[3 + k] >= rel else oracle.ST_DELIVERED
        assert st[5 + k] == want
    assert np.array_equal(rng[0], s)
    delivered = [i for i in range(8) if st[i] == oracle.ST_DELIVERED]
    assert r["event_id"][delivered].tolist() == list(range(5, 5 + len(delivered)))
    assert ctr[0] == 5 + len(delivered)
    # deliver_time = max(now + latency, round_end)
    for i in delivered:
        assert r["deliver_time"][i] == max(t[i] + 5000, 1000)
    assert r["dst_offsets"].tolist() == [0, 0, len(delivered)]


def test_deliver_interleaved_rng_consumers(oracle):
    """Host::random_mut() is one stream shared by send_packet's draw (worker.rs:360)
    and other consumers (getrandom, random.rs:40; socket port choices; host_rngDouble).
    A host's event log -- syscall draws interleaved with sends -- replayed step by
    step must match the round run with per-packet rng_skip counts (sg_packets.rng_skip),
    whatever each packet's status."""
    lat, loss, host_ip, host_row = _tiny_world()
    seeds = [31, 32]
    # per host: ("sys", steps) = a syscall taking `steps` next_u64 steps; ("send", dst, payload, time)
    log = {0: [("sys", 3), ("send", 200, 10, 100), ("send", 999, 10, 110), ("sys", 1), ("sys", 2),
               ("send", 200, 10, 120), ("send", 200, 10, 20_000), ("sys", 4), ("send", 200, 0, 130)],
           1: [("send", 100, 10, 100), ("sys", 7), ("send", 100, 10, 140), ("send", 200, 10, 150)]}
    sim_end = 10_000
    src, dst, pay, t, skip = [], [], [], [], []
    want_st = []
    rel = {(0, 1): float(np.float32(1) - np.float32(0.5)), (1, 0): float(np.float32(1) - np.float32(0.5)),
           (0, 0): 1.0, (1, 1): 1.0}
    model = {h: oracle.xoshiro_seed(seeds[h]) for h in log}
    ip_host = {100: 0, 200: 1}
    for h, events in log.items():
        pending = 0
        for ev in events:
            if ev[0] == "sys":
                pending += ev[1]
                for _ in range(ev[1]):
                    oracle.xoshiro_next_u64(model[h])
                continue
            _, d, p, tt = ev
            src.append(h), dst.append(d), pay.append(p), t.append(tt), skip.append(pending)
            pending = 0
            if tt >= sim_end:
                want_st.append(oracle.ST_SIM_END)
            elif d not in ip_host:
                want_st.append(oracle.ST_DROP_NO_DST)
            else:
                chance = oracle.xoshiro_next_f64(model[h])
                drop = chance >= rel[(h, ip_host[d])] and p > 0
                want_st.append(oracle.ST_DROP_LOSS if drop else oracle.ST_DELIVERED)
        # trailing syscall draws after the host's last send stay with the CPU (sg_hosts_skip carries them)
    rng = np.stack([oracle.xoshiro_seed(s_) for s_ in seeds])
    ctr = np.zeros(2, np.uint64)
    r = oracle.deliver_round(1000, sim_end, 0, src, dst, pay, t, host_ip, host_row, lat, loss, rng, ctr,
                             rng_skip=skip)
    assert r["status"].tolist() == want_st
    for h in log:
        tail = 0
        for ev in reversed(log[h]):
            if ev[0] != "sys":
                break
            tail += ev[1]
        s_ = rng[h].copy()
        for _ in range(tail):
            oracle.xoshiro_next_u64(s_)
        assert np.array_equal(s_, model[h]), h
    # no skips = the plain round
    rng0 = np.stack([oracle.xoshiro_seed(s_) for s_ in seeds])
    a = oracle.deliver_round(1000, sim_end, 0, src, dst, pay, t, host_ip, host_row, lat, loss, rng0.copy(),
                             np.zeros(2, np.uint64), rng_skip=[0] * len(src))
    b = oracle.deliver_round(1000, sim_end, 0, src, dst, pay, t, host_ip, host_row, lat, loss, rng0.copy(),
                             np.zeros(2, np.uint64))
    assert np.array_equal(a["status"], b["status"]) and np.array_equal(a["deliver_time"], b["deliver_time"])


def test_deliver_bootstrap_and_order(oracle):
    lat, loss, host_ip, host_row = _tiny_world()
    loss[:] = 1.0  # everything would drop ...
    rng = np.stack([oracle.xoshiro_seed(1), oracle.xoshiro_seed(2)])
    ctr = np.zeros(2, np.uint64)
    src = [0, 0, 1, 1]
    dst = [200, 100, 100, 100]
    t = [10, 20, 10, 10]
    # ... but not while bootstrapping (worker.rs:327-328, 365)
    r = oracle.deliver_round(100_000, 10**12, 50, src, dst, [1] * 4, t, host_ip, host_row, lat, loss, rng, ctr)
    assert (r["status"] == oracle.ST_DELIVERED).all()
    # dst host 0 receives pkt1 (0->0, t=20+1000), pkt2 & pkt3 (1->0, t=10+5000): all clamp to round_end
    b, e = r["dst_offsets"][0], r["dst_offsets"][1]
    assert r["dst_order"][b:e].tolist() == [1, 2, 3]  # equal times: by (src_host, event_id)


@pytest.mark.parametrize("threads", [2, 7, 16])
def test_deliver_round_multithreaded_equals_sequential(oracle, threads):
    """The CPU baseline's multi-threaded restatement (hosts split over threads, per-thread
    destination histograms, parallel per-destination sort) is identical to the sequential one."""
    rng = np.random.default_rng(threads)
    n_nodes = 40
    g = synth.ring_chords_graph(n_nodes, 5.0, seed=threads)
    rc, lat, loss, _ = oracle.shortest_paths(n_nodes, g["src"], g["dst"], g["lat"], g["loss"], False,
                                             np.arange(n_nodes, dtype=np.uint32), threads=4)
    loss = loss.copy()
    loss[::3, ::2] = np.float32(0.25)
    hosts = synth.make_hosts(3000, n_nodes, general_seed=threads, exact_seeds=False)
    t0 = 946684800 * 10**9
    pk = synth.make_packets(50000, hosts, t0, t0 + 10**6, seed=threads, p_unknown_dst=0.01)
    outs = []
    for th in (1, threads):
        r = np.stack([oracle.xoshiro_seed(int(s)) for s in hosts["seed"]]).astype(np.uint64)
        c = np.zeros(len(hosts["seed"]), np.uint64)
        o = oracle.deliver_round(t0 + 10**6, 2**63, t0 + 200_000, pk["src"], pk["dst_ip"], pk["payload"],
                                 pk["send_time"], hosts["ip"], hosts["route"], lat, loss, r, c, threads=th)
        outs.append((o, r, c))
    (a, ra, ca), (b, rb, cb) = outs
    for k in ("status", "deliver_time", "event_id", "dst_order", "dst_offsets"):
        assert np.array_equal(a[k], b[k]), k
    assert (a["delivered"], a["min_deliver"], a["min_lat"]) == (b["delivered"], b["min_deliver"], b["min_lat"])
    assert np.array_equal(ra, rb) and np.array_equal(ca, cb)


@pytest.mark.parametrize("directed", [False, True])
def test_faithful_routing_build_matches_dense(oracle, directed):
    """The reference-cost CPU baseline (SipHash maps, contains filter, global map,
    id remap; sg_faithful.c) builds the same table as the dense restatement."""
    g = synth.ring_chords_graph(300, 6.0, seed=4, directed=directed, parallel=0.02)
    used = np.random.default_rng(4).permutation(300)[:220].astype(np.uint32)
    ids = (np.arange(300) * 7 + 3).astype(np.uint32)
    rc, lat, loss, _ = oracle.shortest_paths(300, g["src"], g["dst"], g["lat"], g["loss"], directed, used, threads=2)
    assert rc == 0
    rc2, flat, floss, ph = oracle.routing_faithful(300, g["src"], g["dst"], g["lat"], g["loss"], directed, used,
                                                   rows=150, node_ids=ids, threads=3)
    assert rc2 == 0 and all(t >= 0 for t in ph)
    assert np.array_equal(flat, lat[:150])
    assert np.array_equal(floss.view(np.uint32), loss[:150].view(np.uint32))


@pytest.mark.parametrize("threads", [1, 3, 8])
def test_faithful_delivery_round_matches_dense(oracle, threads):
    """The reference-cost delivery baseline (sg_faithful.c sgo_deliver_faithful: SipHash
    Dns / IpAssignment / RoutingInfo maps, the locked packet counter, a mutex'd binary
    heap per destination, hosts round-robin over threads) delivers the same round as
    the dense restatement: statuses, times, event ids, queue order, minima, streams."""
    n_nodes = 60
    g = synth.ring_chords_graph(n_nodes, 5.0, seed=7)
    rc, lat, loss, _ = oracle.shortest_paths(n_nodes, g["src"], g["dst"], g["lat"], g["loss"], False,
                                             np.arange(n_nodes, dtype=np.uint32), threads=4)
    assert rc == 0
    loss = loss.copy()
    loss[::4, ::3] = np.float32(0.3)
    hosts = synth.make_hosts(2500, n_nodes, general_seed=3, exact_seeds=False)
    t0 = 946684800 * 10**9
    pk = synth.make_packets(40000, hosts, t0, t0 + 10**6, seed=threads, p_unknown_dst=0.02)
    sim_end = t0 + 10**6 - 5000  # a few packets past the end
    outs = []
    for fn in (oracle.deliver_round, oracle.deliver_faithful):
        r = np.stack([oracle.xoshiro_seed(int(s)) for s in hosts["seed"]]).astype(np.uint64)
        c = np.zeros(len(hosts["seed"]), np.uint64)
        o = fn(t0 + 10**6, sim_end, t0 + 200_000, pk["src"], pk["dst_ip"], pk["payload"], pk["send_time"],
               hosts["ip"], hosts["route"], lat, loss, r, c, threads=threads)
        outs.append((o, r, c))
    (a, ra, ca), (b, rb, cb) = outs
    for k in ("status", "deliver_time", "event_id", "dst_order", "dst_offsets"):
        assert np.array_equal(a[k], b[k]), k
    assert (a["delivered"], a["min_deliver"], a["min_lat"]) == (b["delivered"], b["min_deliver"], b["min_lat"])
    assert np.array_equal(ra, rb) and np.array_equal(ca, cb)
    assert b["setup_s"] > 0 and b["round_s"] > 0
    assert (a["status"] == 3).any() and (a["status"] == 2).any() and (a["status"] == 1).any()


@pytest.mark.parametrize("directed,parallel,wide", [(False, 0.0, False), (True, 0.0, False), (False, 0.2, False),
                                                   (True, 0.3, False), (False, 0.0, True), (True, 0.1, True)])
def test_fixed_point_certificate(oracle, directed, parallel, wide):
    """sgo_check_fixed_point accepts exactly the Dijkstra table: 0 failing cells on the
    restatement's own table (ties, parallel edges, zero-loss runs), and the first failing
    cell of a table changed in one latency, one loss bit, one diagonal, or two rows swapped."""
    g = synth.ring_chords_graph(700, 6.0, seed=11 + int(directed), directed=directed, parallel=parallel,
                                lat_lo_us=1, lat_hi_us=4)  # tiny latency range: many equal-latency paths
    if wide:  # some edges and paths of 2^32 ns and more: the checker's u64 path instead of packed keys
        g["lat"] = g["lat"] * np.where(np.random.default_rng(5).random(len(g["lat"])) < 0.3, 2**31, 1).astype(np.uint64)
    n = g["n"]
    used = np.random.default_rng(3).permutation(n).astype(np.uint32)  # any order of all nodes
    rc, lat, loss, _ = oracle.shortest_paths(n, g["src"], g["dst"], g["lat"], g["loss"], directed, used, threads=4)
    assert rc == 0
    args = (n, g["src"], g["dst"], g["lat"], g["loss"], directed, used)
    assert oracle.check_fixed_point(*args, lat, loss, threads=4) == (0, (2**32 - 1, 2**32 - 1))
    # a row block
    assert oracle.check_fixed_point(*args, lat[100:300].copy(), loss[100:300].copy(), rows=(100, 300))[0] == 0
    cases = []
    l2 = lat.copy(); l2[37, 400] += 1; cases.append((l2, loss, (37, None)))  # (neighbours fail too)
    f2 = loss.copy(); off = 401 if f2[37, 401] > 0 else 402
    f2.view(np.uint32)[37, off] ^= 1; cases.append((lat, f2, (37, None)))
    l3 = lat.copy(); l3[5, 5] += 7; cases.append((l3, loss, (5, 5)))  # the diagonal alone
    l4, f4 = lat.copy(), loss.copy(); l4[[8, 9]] = l4[[9, 8]]; f4[[8, 9]] = f4[[9, 8]]
    cases.append((l4, f4, (8, None)))
    for tl, tf, (r, c) in cases:
        bad, (br, bc) = oracle.check_fixed_point(*args, tl, tf, threads=3)
        assert bad > 0 and br == r and (c is None or bc == c), (bad, br, bc, r, c)


def test_fixed_point_certificate_needs_every_node(oracle):
    g = synth.ring_chords_graph(50, 4.0, seed=2)
    used = np.arange(40, dtype=np.uint32)
    z = np.zeros((40, 40), np.uint64)
    assert oracle.check_fixed_point(50, g["src"], g["dst"], g["lat"], g["loss"], False, used, z,
                                    z.astype(np.float32))[0] == -oracle.ERR_ARG
