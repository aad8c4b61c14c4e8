"""ctypes front end for the CPU oracle (oracle/sg_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
`cpu_baseline` leg of bench.py, never by the product package `shadow_amd`.
Every function cites the reference code it restates (see sg_oracle.c).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libsg_oracle.so")

OK, ERR_NO_EDGE, ERR_MULTI_EDGE, ERR_UNREACHABLE, ERR_OOM, ERR_ARG = range(6)
ST_DELIVERED, ST_DROP_LOSS, ST_DROP_NO_DST, ST_SIM_END = range(4)

_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(
            os.path.join(_HERE, "sg_oracle.c")
        ):
            build()
        L = C.CDLL(_LIB_PATH)
        u32p, u64p, f32p, u8p = (C.POINTER(t) for t in (C.c_uint32, C.c_uint64, C.c_float, C.c_uint8))
        L.sgo_shortest_paths.restype = C.c_int
        L.sgo_shortest_paths.argtypes = [C.c_uint32, C.c_uint32, u32p, u32p, u64p, f32p, C.c_int, u32p,
                                         C.c_uint32, C.c_uint32, C.c_uint32, u64p, f32p, C.c_int, u32p, u32p]
        L.sgo_check_fixed_point.restype = C.c_int64
        L.sgo_check_fixed_point.argtypes = [C.c_uint32, C.c_uint32, u32p, u32p, u64p, f32p, C.c_int, u32p,
                                             C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p, C.c_void_p, C.c_int,
                                             u32p, u32p]
        L.sgo_direct_paths.restype = C.c_int
        L.sgo_direct_paths.argtypes = [C.c_uint32, C.c_uint32, u32p, u32p, u64p, f32p, C.c_int, u32p,
                                       C.c_uint32, u64p, f32p, u32p, u32p]
        L.sgo_path_add.restype = None
        L.sgo_path_add.argtypes = [C.c_uint64, C.c_float, C.c_uint64, C.c_float, u64p, f32p]
        L.sgo_splitmix64_next.restype = C.c_uint64
        L.sgo_splitmix64_next.argtypes = [u64p]
        L.sgo_xoshiro_seed_from_u64.restype = None
        L.sgo_xoshiro_seed_from_u64.argtypes = [C.c_uint64, u64p]
        L.sgo_xoshiro_next_u64.restype = C.c_uint64
        L.sgo_xoshiro_next_u64.argtypes = [u64p]
        L.sgo_xoshiro_next_f64.restype = C.c_double
        L.sgo_xoshiro_next_f64.argtypes = [u64p]
        L.sgo_siphash13.restype = C.c_uint64
        L.sgo_siphash13.argtypes = [C.c_char_p, C.c_size_t]
        L.sgo_host_seed.restype = C.c_uint64
        L.sgo_host_seed.argtypes = [C.c_uint64, C.c_char_p, C.c_size_t]
        L.sgo_smallest_latency.restype = C.c_uint64
        L.sgo_smallest_latency.argtypes = [u64p, C.c_size_t]
        L.sgo_deliver_round.restype = C.c_int64
        L.sgo_codel_control_law.argtypes = [C.c_uint64, C.c_uint64]
        L.sgo_codel_control_law.restype = C.c_uint64
        L.sgo_codel_run.argtypes = [C.c_uint32, C.c_uint32] + [C.c_void_p] * 11 + [C.c_uint32] + [C.c_void_p] * 7 + [
            C.c_uint32]
        L.sgo_codel_run.restype = C.c_int
        L.sgo_token_bucket_remove.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.POINTER(C.c_uint64)]
        L.sgo_token_bucket_remove.restype = C.c_int
        L.sgo_inbound_run.argtypes = [C.c_uint32, C.c_uint32] + [C.c_void_p] * 21 + [C.c_uint32] + \
            [C.c_void_p] * 4 + [C.c_uint64] * 3 + [C.c_void_p] * 3 + [C.c_uint32]
        L.sgo_inbound_run.restype = C.c_int
        L.sgo_outbound_run.argtypes = [C.c_uint32, C.c_uint32] + [C.c_void_p] * 15 + [C.c_uint32] + \
            [C.c_void_p] * 8 + [C.c_uint64] * 3 + [C.c_void_p] * 3 + [C.c_uint32] + [C.c_void_p] * 5 + \
            [C.c_uint32, C.c_void_p]
        L.sgo_outbound_run.restype = C.c_int
        # the multi-threaded baselines: the same arguments and a thread count (outbound: + out_group)
        L.sgo_codel_run_mt.argtypes = L.sgo_codel_run.argtypes + [C.c_uint32]
        L.sgo_codel_run_mt.restype = C.c_int
        L.sgo_inbound_run_mt.argtypes = L.sgo_inbound_run.argtypes + [C.c_uint32]
        L.sgo_inbound_run_mt.restype = C.c_int
        L.sgo_outbound_run_mt.argtypes = L.sgo_outbound_run.argtypes + [C.c_void_p, C.c_uint32]
        L.sgo_outbound_run_mt.restype = C.c_int
        L.sgo_deliver_round_mt.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint32] + [C.c_void_p] * 4 + [
            C.c_uint32, C.c_void_p, C.c_void_p, C.c_uint32] + [C.c_void_p] * 11 + [C.c_int]
        L.sgo_deliver_round_mt.restype = C.c_int64
        L.sgo_deliver_faithful.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint32] + [C.c_void_p] * 4 + [
            C.c_uint32, C.c_void_p, C.c_void_p, C.c_uint32] + [C.c_void_p] * 11 + [C.c_int, C.c_void_p, C.c_void_p]
        L.sgo_deliver_faithful.restype = C.c_int64
        L.sgo_deliver_round.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint32, u32p, u32p, u32p, u64p,
                                        C.c_uint32, u32p, u32p, C.c_uint32, u64p, f32p, u64p, u64p, u8p, u64p,
                                        u64p, u32p, u32p, u64p, u64p, C.c_void_p]
        _lib = L
    return _lib


def _p(a: np.ndarray, t):
    return a.ctypes.data_as(C.POINTER(t))


def _arr(x, dtype):
    return np.ascontiguousarray(np.asarray(x, dtype=dtype))


def path_add(a_lat, a_loss, b_lat, b_loss):
    """PathProperties + PathProperties (graph/mod.rs:322-331)."""
    ol, of = C.c_uint64(), C.c_float()
    lib().sgo_path_add(a_lat, a_loss, b_lat, b_loss, C.byref(ol), C.byref(of))
    return ol.value, np.float32(of.value)


def shortest_paths(n_nodes, src, dst, lat, loss, directed, used, rows=None, threads=1):
    """NetworkGraph::compute_shortest_paths (graph/mod.rs:183-228), dense output.

    Returns (rc, lat[rows x n_used] u64, loss[rows x n_used] f32, (err_row, err_col)).
    """
    src, dst = _arr(src, np.uint32), _arr(dst, np.uint32)
    lat, loss = _arr(lat, np.uint64), _arr(loss, np.float32)
    used = _arr(used, np.uint32)
    nu = len(used)
    r0, r1 = (0, nu) if rows is None else rows
    out_lat = np.zeros((r1 - r0, nu), np.uint64)
    out_loss = np.zeros((r1 - r0, nu), np.float32)
    ea, eb = C.c_uint32(0), C.c_uint32(0)
    rc = lib().sgo_shortest_paths(n_nodes, len(src), _p(src, C.c_uint32), _p(dst, C.c_uint32),
                                  _p(lat, C.c_uint64), _p(loss, C.c_float), int(bool(directed)),
                                  _p(used, C.c_uint32), nu, r0, r1, _p(out_lat, C.c_uint64),
                                  _p(out_loss, C.c_float), threads, C.byref(ea), C.byref(eb))
    return rc, out_lat, out_loss, (ea.value, eb.value)


def check_fixed_point(n_nodes, src, dst, lat, loss, directed, used, tab_lat, tab_loss, rows=None, threads=1):
    """Whole-table certificate (sg_oracle.c sgo_check_fixed_point): the number of cells of the
    given rows [r0, r1) (tab_lat u64 / tab_loss f32, (r1 - r0) x n_used, row-major, any object
    exposing a C-contiguous buffer) that break compute_shortest_paths' fixed-point equations
    (graph/mod.rs:183-228), 0 when the rows are the reference's table bit for bit; and the first
    failing (row, col).  Every node must be used."""
    src, dst = _arr(src, np.uint32), _arr(dst, np.uint32)
    lat, loss = _arr(lat, np.uint64), _arr(loss, np.float32)
    used = _arr(used, np.uint32)
    nu = len(used)
    r0, r1 = (0, nu) if rows is None else rows
    tl, tf = np.asarray(tab_lat), np.asarray(tab_loss)
    assert tl.dtype.itemsize == 8 and tf.dtype.itemsize == 4 and tl.size == tf.size == (r1 - r0) * nu
    assert tl.flags.c_contiguous and tf.flags.c_contiguous
    br, bc = C.c_uint32(0), C.c_uint32(0)
    bad = lib().sgo_check_fixed_point(n_nodes, len(src), _p(src, C.c_uint32), _p(dst, C.c_uint32),
                                      _p(lat, C.c_uint64), _p(loss, C.c_float), int(bool(directed)),
                                      _p(used, C.c_uint32), nu, r0, r1, tl.ctypes.data, tf.ctypes.data, threads,
                                      C.byref(br), C.byref(bc))
    return int(bad), (br.value, bc.value)


def routing_faithful(n_nodes, src, dst, lat, loss, directed, used, rows=None, node_ids=None, threads=1,
                     read_back=True):
    """The reference's routing build cost for cost (sg_faithful.c): petgraph-style
    Dijkstra with a SipHash score map, the nodes.contains filter, per-source and
    global HashMaps, the self-loop override and the id remap (graph/mod.rs:183-228,
    sim_config.rs:411-448), for source rows [0, rows).  Returns (rc, lat, loss,
    phase seconds [dijkstra+filter+per-source maps, global collect, self pairs, remap])."""
    src, dst = _arr(src, np.uint32), _arr(dst, np.uint32)
    lat, loss = _arr(lat, np.uint64), _arr(loss, np.float32)
    used = _arr(used, np.uint32)
    nu = len(used)
    k = nu if rows is None else int(rows)
    ids = _arr(np.arange(n_nodes) if node_ids is None else node_ids, np.uint32)
    out_lat = np.zeros((k, nu), np.uint64) if read_back else None
    out_loss = np.zeros((k, nu), np.float32) if read_back else None
    ph = (C.c_double * 4)()
    rc = lib().sgo_routing_faithful(n_nodes, len(src), _p(src, C.c_uint32), _p(dst, C.c_uint32),
                                    _p(lat, C.c_uint64), _p(loss, C.c_float), int(bool(directed)),
                                    _p(used, C.c_uint32), nu, k, _p(ids, C.c_uint32), int(threads), ph,
                                    _p(out_lat, C.c_uint64) if read_back else None,
                                    _p(out_loss, C.c_float) if read_back else None)
    return rc, out_lat, out_loss, list(ph)


def direct_paths(n_nodes, src, dst, lat, loss, directed, used):
    """NetworkGraph::get_direct_paths (graph/mod.rs:230-252), dense output."""
    src, dst = _arr(src, np.uint32), _arr(dst, np.uint32)
    lat, loss = _arr(lat, np.uint64), _arr(loss, np.float32)
    used = _arr(used, np.uint32)
    nu = len(used)
    out_lat = np.zeros((nu, nu), np.uint64)
    out_loss = np.zeros((nu, nu), np.float32)
    ea, eb = C.c_uint32(0), C.c_uint32(0)
    rc = lib().sgo_direct_paths(n_nodes, len(src), _p(src, C.c_uint32), _p(dst, C.c_uint32),
                                _p(lat, C.c_uint64), _p(loss, C.c_float), int(bool(directed)),
                                _p(used, C.c_uint32), nu, _p(out_lat, C.c_uint64), _p(out_loss, C.c_float),
                                C.byref(ea), C.byref(eb))
    return rc, out_lat, out_loss, (ea.value, eb.value)


def xoshiro_seed(seed: int) -> np.ndarray:
    """Xoshiro256PlusPlus::seed_from_u64 (SplitMix64; sim_config.rs:48-51, host.rs:221)."""
    s = np.zeros(4, np.uint64)
    lib().sgo_xoshiro_seed_from_u64(seed, _p(s, C.c_uint64))
    return s


def xoshiro_next_u64(state: np.ndarray) -> int:
    return lib().sgo_xoshiro_next_u64(_p(state, C.c_uint64))


def xoshiro_next_f64(state: np.ndarray) -> float:
    """rand 0.9 `random::<f64>()` on the host stream (worker.rs:360)."""
    return lib().sgo_xoshiro_next_f64(_p(state, C.c_uint64))


def siphash13(data: bytes) -> int:
    return lib().sgo_siphash13(data, len(data))


def host_seed(general_seed: int, hostname: str) -> int:
    """HostInfo.seed (sim_config.rs:50-54,221-225,242). Parity unpinned (std SipHash)."""
    b = hostname.encode()
    return lib().sgo_host_seed(general_seed, b, len(b))


def smallest_latency(lat: np.ndarray) -> int:
    lat = _arr(lat, np.uint64).ravel()
    return lib().sgo_smallest_latency(_p(lat, C.c_uint64), lat.size)


def deliver_round(round_end, sim_end, bootstrap_end, src_host, dst_ip, payload_len, send_time,
                  host_ip, host_row, tab_lat, tab_loss, rng, event_ctr, threads: int = 1, rng_skip=None):
    """Worker::send_packet over a round's batch (worker.rs:322-397) + event order (event.rs:84-155).

    rng (H x 4 u64) and event_ctr (H u64) are updated in place.  rng_skip (per
    packet, optional): steps the source host's other RNG consumers take before the
    packet (sg_oracle.c sgo_deliver_round; runs single-threaded).
    Returns dict(status, deliver_time, event_id, dst_order, dst_offsets, min_deliver, min_lat, delivered).
    """
    src_host, dst_ip = _arr(src_host, np.uint32), _arr(dst_ip, np.uint32)
    payload_len, send_time = _arr(payload_len, np.uint32), _arr(send_time, np.uint64)
    host_ip, host_row = _arr(host_ip, np.uint32), _arr(host_row, np.uint32)
    tab_lat, tab_loss = _arr(tab_lat, np.uint64), _arr(tab_loss, np.float32)
    assert rng.dtype == np.uint64 and rng.flags.c_contiguous and event_ctr.dtype == np.uint64
    n, H = len(src_host), len(host_ip)
    ncols = tab_lat.shape[-1]
    status = np.zeros(n, np.uint8)
    deliver = np.zeros(n, np.uint64)
    eid = np.zeros(n, np.uint64)
    order = np.zeros(max(n, 1), np.uint32)
    offs = np.zeros(H + 1, np.uint32)
    mind, minl = C.c_uint64(), C.c_uint64()
    skip = None if rng_skip is None else _arr(rng_skip, np.uint32)
    if skip is not None:
        assert len(skip) == n
        threads = 1
    if threads > 1:  # the multi-threaded restatement (same results; packets grouped by source host)
        v = lambda a: a.ctypes.data_as(C.c_void_p)
        nd = lib().sgo_deliver_round_mt(round_end, sim_end, bootstrap_end, n, v(src_host), v(dst_ip), v(payload_len),
                                        v(send_time), H, v(host_ip), v(host_row), ncols, v(tab_lat), v(tab_loss),
                                        v(rng), v(event_ctr), v(status), v(deliver), v(eid), v(order), v(offs),
                                        C.byref(mind), C.byref(minl), int(threads))
        if nd == -2:
            raise OverflowError("send time + latency overflows EmulatedTime (emulated_time.rs:121-126 panics)")
        if nd < 0:
            raise ValueError("sgo_deliver_round_mt: bad argument")
        return dict(status=status, deliver_time=deliver, event_id=eid, dst_order=order[:nd],
                    dst_offsets=offs, min_deliver=mind.value, min_lat=minl.value, delivered=int(nd))
    nd = lib().sgo_deliver_round(round_end, sim_end, bootstrap_end, n, _p(src_host, C.c_uint32),
                                 _p(dst_ip, C.c_uint32), _p(payload_len, C.c_uint32), _p(send_time, C.c_uint64),
                                 H, _p(host_ip, C.c_uint32), _p(host_row, C.c_uint32), ncols,
                                 _p(tab_lat, C.c_uint64), _p(tab_loss, C.c_float), _p(rng, C.c_uint64),
                                 _p(event_ctr, C.c_uint64), _p(status, C.c_uint8), _p(deliver, C.c_uint64),
                                 _p(eid, C.c_uint64), _p(order, C.c_uint32), _p(offs, C.c_uint32),
                                 C.byref(mind), C.byref(minl), None if skip is None else skip.ctypes.data)
    if nd == -2:
        raise OverflowError("send time + latency overflows EmulatedTime (emulated_time.rs:121-126 panics)")
    if nd < 0:
        raise ValueError("sgo_deliver_round: bad argument")
    return dict(status=status, deliver_time=deliver, event_id=eid, dst_order=order[:nd],
                dst_offsets=offs, min_deliver=mind.value, min_lat=minl.value, delivered=int(nd))


def deliver_faithful(round_end, sim_end, bootstrap_end, src_host, dst_ip, payload_len, send_time,
                     host_ip, host_node, tab_lat, tab_loss, rng, event_ctr, threads: int = 1):
    """The reference's delivery round cost for cost (sg_faithful.c sgo_deliver_faithful):
    Worker::send_packet with SipHash Dns / IpAssignment / RoutingInfo lookups, the
    global RwLock'd packet counter and a mutex'd binary heap per destination queue,
    hosts round-robin over `threads` workers.  host_node[h] = host h's node, a row and
    column of the n x n table.  rng / event_ctr are updated in place.  Returns the
    deliver_round dict plus setup_s (building the maps) and round_s (the round)."""
    src_host, dst_ip = _arr(src_host, np.uint32), _arr(dst_ip, np.uint32)
    payload_len, send_time = _arr(payload_len, np.uint32), _arr(send_time, np.uint64)
    host_ip, host_node = _arr(host_ip, np.uint32), _arr(host_node, np.uint32)
    tab_lat, tab_loss = _arr(tab_lat, np.uint64), _arr(tab_loss, np.float32)
    assert rng.dtype == np.uint64 and rng.flags.c_contiguous and event_ctr.dtype == np.uint64
    n, H = len(src_host), len(host_ip)
    nn = tab_lat.shape[-1]
    assert tab_lat.size == nn * nn
    status, deliver, eid = np.zeros(n, np.uint8), np.zeros(n, np.uint64), np.zeros(n, np.uint64)
    order, offs = np.zeros(max(n, 1), np.uint32), np.zeros(H + 1, np.uint32)
    mind, minl, ts, tr = C.c_uint64(), C.c_uint64(), C.c_double(), C.c_double()
    v = lambda a: a.ctypes.data_as(C.c_void_p)
    nd = lib().sgo_deliver_faithful(round_end, sim_end, bootstrap_end, n, v(src_host), v(dst_ip), v(payload_len),
                                    v(send_time), H, v(host_ip), v(host_node), nn, v(tab_lat), v(tab_loss), v(rng),
                                    v(event_ctr), v(status), v(deliver), v(eid), v(order), v(offs), C.byref(mind),
                                    C.byref(minl), int(threads), C.byref(ts), C.byref(tr))
    if nd == -2:
        raise OverflowError("send time + latency overflows EmulatedTime (emulated_time.rs:121-126 panics)")
    if nd < 0:
        raise ValueError("sgo_deliver_faithful: bad argument")
    return dict(status=status, deliver_time=deliver, event_id=eid, dst_order=order[:nd], dst_offsets=offs,
                min_deliver=mind.value, min_lat=minl.value, delivered=int(nd), setup_s=ts.value, round_s=tr.value)


# ---------------------------------------------------------------------------
# Router inbound CoDel queue (router/codel_queue.rs), one per host
# ---------------------------------------------------------------------------
CODEL_TARGET_NS = 10_000_000      # codel_queue.rs:23
CODEL_INTERVAL_NS = 100_000_000   # codel_queue.rs:28
CODEL_MTU = 1500                  # definitions.h:124
CD_DROP, CD_HAS_IEND, CD_HAS_DNEXT = 1, 2, 4
CD_PUSH, CD_POP = 0, 1
CD_NONE = 0xFFFFFFFF


def codel_control_law(t: int, count: int) -> int:
    """apply_control_law (codel_queue.rs:285-298)."""
    return int(lib().sgo_codel_control_law(t, count))


def codel_state(n_hosts: int, cap: int) -> dict:
    """Empty queues (CoDelQueue::new, codel_queue.rs:85-95) in the ring layout the HIP side uses."""
    return dict(cap=cap, flags=np.zeros(n_hosts, np.uint8), interval_end=np.zeros(n_hosts, np.uint64),
                drop_next=np.zeros(n_hosts, np.uint64), cur=np.zeros(n_hosts, np.uint64),
                prev=np.zeros(n_hosts, np.uint64), bytes=np.zeros(n_hosts, np.uint64),
                head=np.zeros(n_hosts, np.uint32), tail=np.zeros(n_hosts, np.uint32),
                ring_pkt=np.zeros(n_hosts * cap, np.uint32), ring_ts=np.zeros(n_hosts * cap, np.uint64),
                ring_len=np.zeros(n_hosts * cap, np.uint32))


def codel_run(state: dict, host, kind, time, pkt, length, pkt_status: np.ndarray, threads: int = 1) -> np.ndarray:
    """Push/pop events (grouped by ascending host, each host's in order) through the
    per-host queues; state and pkt_status (1 dequeued, 2 dropped) updated in place.
    Returns pop_result (the popped packet, or CD_NONE; CD_NONE for pushes).  threads > 1:
    hosts dealt round-robin over that many threads (sgo_codel_run_mt), the same results."""
    host, kind = _arr(host, np.uint32), _arr(kind, np.uint8)
    time, pkt, length = _arr(time, np.uint64), _arr(pkt, np.uint32), _arr(length, np.uint32)
    n = len(host)
    res = np.zeros(max(n, 1), np.uint32)
    H = len(state["flags"])
    v = lambda a: a.ctypes.data_as(C.c_void_p)
    args = (H, state["cap"], v(state["flags"]), v(state["interval_end"]), v(state["drop_next"]), v(state["cur"]),
            v(state["prev"]), v(state["bytes"]), v(state["head"]), v(state["tail"]), v(state["ring_pkt"]),
            v(state["ring_ts"]), v(state["ring_len"]), n, v(host), v(kind), v(time), v(pkt), v(length), v(res),
            v(pkt_status), len(pkt_status))
    rc = lib().sgo_codel_run_mt(*args, int(threads)) if threads > 1 else lib().sgo_codel_run(*args)
    if rc:
        raise ValueError(f"sgo_codel_run: error {rc}")
    return res[:n]


# ---------------------------------------------------------------------------
# Inbound pipeline: router CoDel queue -> relay_inet_in token bucket
# ---------------------------------------------------------------------------
RL_PENDING, RL_NEVER, RL_CACHED = 1, 2, 4
TB_INTERVAL_NS = 1_000_000   # relay/mod.rs:297


def token_bucket_remove(state: np.ndarray, dec: int, now: int):
    """TokenBucket::conforming_remove_inner on state = u64[5] {capacity, balance,
    refill_increment, last_refill, refill_interval}: (True, balance) or (False, wait)."""
    assert state.dtype == np.uint64 and len(state) == 5
    w = C.c_uint64()
    ok = lib().sgo_token_bucket_remove(state.ctypes.data_as(C.c_void_p), dec, now, C.byref(w))
    return (True, int(state[1])) if ok else (False, int(w.value))


def inbound_state(bw_down_bits: np.ndarray, cap: int, t0: int = 946684800 * 10**9) -> dict:
    """Empty router queues + Idle relays with full buckets (Relay::new / create_token_bucket,
    relay/mod.rs:296-309: refill max(1, B/1000) bytes per 1 ms, capacity refill + MTU)."""
    n = len(bw_down_bits)
    st = codel_state(n, cap)
    refill = np.maximum(1, (np.asarray(bw_down_bits, np.uint64) // np.uint64(8)) // np.uint64(1000)).astype(np.uint64)
    st.update(rflags=np.zeros(n, np.uint8), task_time=np.zeros(n, np.uint64), task_id=np.zeros(n, np.uint64),
              task_born=np.zeros(n, np.uint64), cached_pkt=np.zeros(n, np.uint32),
              cached_len=np.zeros(n, np.uint32), tb_cap=refill + np.uint64(CODEL_MTU), tb_bal=refill + np.uint64(CODEL_MTU),
              tb_inc=refill, tb_last=np.full(n, t0, np.uint64))
    return st


def inbound_run(st: dict, host, time, pkt, length, window_end: int, bootstrap_end: int, sim_end: int,
                event_ctr: np.ndarray, fwd_time: np.ndarray, pkt_status: np.ndarray, threads: int = 1) -> None:
    host, time = _arr(host, np.uint32), _arr(time, np.uint64)
    pkt, length = _arr(pkt, np.uint32), _arr(length, np.uint32)
    v = lambda a: a.ctypes.data_as(C.c_void_p)
    H = len(st["flags"])
    args = (H, st["cap"], *[v(st[k]) for k in (
        "flags", "interval_end", "drop_next", "cur", "prev", "bytes", "head", "tail", "ring_pkt", "ring_ts",
        "ring_len", "rflags", "task_time", "task_id", "task_born", "cached_pkt", "cached_len", "tb_cap", "tb_bal", "tb_inc", "tb_last")],
        len(host), v(host), v(time), v(pkt), v(length), window_end, bootstrap_end, sim_end, v(event_ctr),
        v(fwd_time), v(pkt_status), len(pkt_status))
    rc = lib().sgo_inbound_run_mt(*args, int(threads)) if threads > 1 else lib().sgo_inbound_run(*args)
    if rc:
        raise ValueError(f"sgo_inbound_run: error {rc}")


# Outbound pipeline: interface FIFO -> relay_inet_out -> router -> send_packet
def outbound_state(host_ipv4, bw_up_bits: np.ndarray, cap: int, t0: int = 946684800 * 10**9) -> dict:
    """Empty interface queues + Idle relays with full buckets (Relay::new / create_token_bucket,
    relay/mod.rs:91-109, :278-319).  `cap` is rounded up to a power of two like the library's."""
    n = len(bw_up_bits)
    c = 1
    while c < cap:
        c <<= 1
    refill = np.maximum(1, (np.asarray(bw_up_bits, np.uint64) // np.uint64(8)) // np.uint64(1000)).astype(np.uint64)
    return dict(cap=c, host_ip=np.ascontiguousarray(host_ipv4, np.uint32), head=np.zeros(n, np.uint32),
                tail=np.zeros(n, np.uint32), ring_pkt=np.zeros(n * c, np.uint32), ring_len=np.zeros(n * c, np.uint32),
                ring_dst=np.zeros(n * c, np.uint32), ring_pay=np.zeros(n * c, np.uint32),
                rflags=np.zeros(n, np.uint8), task_time=np.zeros(n, np.uint64), task_id=np.zeros(n, np.uint64),
                task_born=np.zeros(n, np.uint64), tb_cap=refill + np.uint64(CODEL_MTU),
                tb_bal=refill + np.uint64(CODEL_MTU), tb_inc=refill, tb_last=np.full(n, t0, np.uint64))


def outbound_run(st: dict, host, time, pkt, length, payload, dst, window_end: int, bootstrap_end: int,
                 sim_end: int, event_ctr: np.ndarray, fwd_time: np.ndarray, pkt_status: np.ndarray,
                 event_id=None, event_created=None, threads: int = 1) -> dict:
    """One window of sends (sgo_outbound_run).  Returns the packets handed to send_packet, in order.
    event_id / event_created (optional, together): the sending event's id (UINT64_MAX: a Packet
    event) and creation time, which order a send against a forward task at the same time.
    threads > 1 (sgo_outbound_run_mt): hosts round-robin over the threads; the packets come
    grouped by thread (hosts ascending within one), a stable sort by src_host restores the order."""
    host, time = _arr(host, np.uint32), _arr(time, np.uint64)
    assert (event_id is None) == (event_created is None)
    eid = None if event_id is None else _arr(event_id, np.uint64)
    eborn = None if event_created is None else _arr(event_created, np.uint64)
    pkt, length, payload, dst = (_arr(x, np.uint32) for x in (pkt, length, payload, dst))
    v = lambda a: a.ctypes.data_as(C.c_void_p)
    H = len(st["head"])
    cap_out = len(host) + int((st["tail"] - st["head"]).astype(np.uint64).sum()) + H
    out = dict(src_host=np.zeros(cap_out, np.uint32), dst_ipv4=np.zeros(cap_out, np.uint32),
               payload_len=np.zeros(cap_out, np.uint32), send_time=np.zeros(cap_out, np.uint64),
               packet=np.zeros(cap_out, np.uint32))
    n_out = C.c_uint32()
    args = (H, st["cap"], *[v(st[k]) for k in (
        "host_ip", "head", "tail", "ring_pkt", "ring_len", "ring_dst", "ring_pay", "rflags", "task_time", "task_id",
        "task_born", "tb_cap", "tb_bal", "tb_inc", "tb_last")], len(host), v(host), v(time), v(pkt), v(length),
        v(payload), v(dst), None if eid is None else v(eid), None if eborn is None else v(eborn), window_end, bootstrap_end, sim_end, v(event_ctr), v(fwd_time), v(pkt_status), len(pkt_status),
        *[v(out[k]) for k in ("src_host", "dst_ipv4", "payload_len", "send_time", "packet")], cap_out, C.byref(n_out))
    if threads > 1:
        rc = lib().sgo_outbound_run_mt(*args, None, int(threads))
    else:
        rc = lib().sgo_outbound_run(*args)
    if rc:
        raise ValueError(f"sgo_outbound_run: error {rc}")
    return {k: a[:n_out.value] for k, a in out.items()}
