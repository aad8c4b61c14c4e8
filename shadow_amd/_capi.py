"""ctypes binding of include/shadow_gpu.h (libshadow_gpu.so, built in-tree).

The product path has no CPU fallback: if the HIP library is missing or fails
to load, importing a compute entry point raises `ShadowGpuUnavailable`.
"""
from __future__ import annotations

import ctypes as C
import os

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_PKG, "libshadow_gpu.so")
HEADER_PATH = os.path.join(os.path.dirname(_PKG), "include", "shadow_gpu.h")

# sg_status (include/shadow_gpu.h)
SG_OK = 0
SG_ABI_VERSION = 7  # include/shadow_gpu.h
SG_ERR_NO_EDGE = 1
SG_ERR_MULTI_EDGE = 2
SG_ERR_UNREACHABLE = 3
SG_ERR_OOM = 4
SG_ERR_INVALID_ARG = 5
SG_ERR_DEVICE = 6
SG_ERR_PARSE = 7
SG_ERR_UNSORTED = 8
SG_ERR_DUPLICATE_IP = 9
SG_ERR_CAPACITY = 10
SG_ERR_TIME_OVERFLOW = 11
SG_ERR_UNSUPPORTED = 12
SG_COMM_ID_BYTES = 128

SG_ROUTE_SHORTEST_PATH = 0x1
SG_ROUTE_OUT_DEVICE = 0x2

SG_PKT_DELIVERED, SG_PKT_DROP_LOSS, SG_PKT_DROP_NO_DST, SG_PKT_SIM_END = range(4)

EXPORTED = [
    "sg_abi_version", "sg_ctx_create", "sg_ctx_destroy", "sg_ctx_set_stream", "sg_ctx_stream",
    "sg_ctx_synchronize", "sg_ctx_last_error", "sg_ctx_last_error_pair", "sg_ctx_enable_timers",
    "sg_ctx_read_timer", "sg_gml_parse", "sg_gml_parse_threads", "sg_gml_load", "sg_gml_graph",
    "sg_gml_node_index", "sg_gml_destroy", "sg_net_create", "sg_net_destroy", "sg_routing_build",
    "sg_routing_min_latency", "sg_hosts_create", "sg_hosts_get_state", "sg_hosts_set_state", "sg_hosts_skip",
    "sg_hosts_destroy", "sg_deliver_round", "sg_deliver_source", "sg_deliver_bucket",
    "sg_deliver_source_padded", "sg_deliver_bucket_padded", "sg_deliver_pad_to_compact",
    "sg_table_pack", "sg_codel_create", "sg_codel_destroy", "sg_codel_run", "sg_codel_ring_cap",
    "sg_codel_get_state", "sg_codel_set_state", "sg_inbound_create", "sg_inbound_destroy", "sg_inbound_ring_cap",
    "sg_inbound_run", "sg_inbound_run_ordered", "sg_ctx_set_packet_counters", "sg_inbound_get_state", "sg_hosts_event_ctr", "sg_outbound_create", "sg_outbound_destroy",
    "sg_outbound_ring_cap", "sg_outbound_run", "sg_outbound_get_state",
    "sg_routing_info_create", "sg_routing_info_destroy", "sg_routing_info_fill", "sg_routing_info_set_rows",
    "sg_routing_info_view", "sg_routing_info_rows", "sg_routing_info_index", "sg_routing_info_path", "sg_routing_info_smallest_latency",
    "sg_routing_info_increment_packet_count", "sg_routing_info_packet_count", "sg_routing_info_set_addresses",
    "sg_worker_get_latency", "sg_worker_get_reliability", "sg_worker_is_routable",
    "sg_comm_unique_id", "sg_comm_create", "sg_comm_destroy", "sg_comm_allgather_rows", "sg_comm_exchange_padded",
    "sg_comm_alltoallv_records", "sg_comm_allgather_u64",
]


class ShadowGpuUnavailable(RuntimeError):
    pass


class ShadowGpuError(RuntimeError):
    """A non-OK sg_status.  `pair` = (row, col) of the failing entry where relevant."""

    def __init__(self, code: int, message: str, pair=(0, 0)):
        super().__init__(message)
        self.code = code
        self.pair = pair


class sg_graph(C.Structure):
    _fields_ = [("n_nodes", C.c_uint32), ("n_edges", C.c_uint32),
                ("edge_src", C.POINTER(C.c_uint32)), ("edge_dst", C.POINTER(C.c_uint32)),
                ("edge_latency_ns", C.POINTER(C.c_uint64)), ("edge_packet_loss", C.POINTER(C.c_float)),
                ("node_gml_id", C.POINTER(C.c_uint32)), ("directed", C.c_uint8)]


class sg_table(C.Structure):
    _fields_ = [("latency_ns", C.c_void_p), ("packet_loss", C.c_void_p), ("n_cols", C.c_uint32),
                ("row_begin", C.c_uint32), ("n_rows", C.c_uint32), ("path_key", C.c_void_p)]


class sg_codel_events(C.Structure):
    _fields_ = [("n_events", C.c_uint32), ("host", C.c_void_p), ("kind", C.c_void_p), ("time_ns", C.c_void_p),
                ("packet", C.c_void_p), ("len", C.c_void_p)]


class sg_codel_state(C.Structure):
    _fields_ = [(k, C.c_void_p) for k in ("flags", "interval_end", "drop_next", "cur_drops", "prev_drops", "bytes",
                                          "head", "tail", "ring_packet", "ring_time", "ring_len")]


class sg_inbound_arrivals(C.Structure):
    _fields_ = [("n", C.c_uint32), ("host", C.c_void_p), ("time_ns", C.c_void_p), ("packet", C.c_void_p),
                ("len", C.c_void_p)]


class sg_inbound_relay_state(C.Structure):
    _fields_ = [(k, C.c_void_p) for k in ("flags", "task_time", "cached_packet", "cached_len", "tb_capacity",
                                          "tb_balance", "tb_increment", "tb_last_refill", "task_event_id",
                                          "task_created_ns")]


class sg_outbound_sends(C.Structure):
    _fields_ = [("n", C.c_uint32)] + [(k, C.c_void_p) for k in ("host", "time_ns", "packet", "len", "payload_len",
                                                                  "dst_ipv4", "event_id", "event_created_ns")]


class sg_outbound_sent(C.Structure):
    _fields_ = [("cap", C.c_uint32)] + [(k, C.c_void_p) for k in ("src_host", "dst_ipv4", "payload_len",
                                                                    "send_time_ns", "packet")]


class sg_outbound_queue_state(C.Structure):
    _fields_ = [(k, C.c_void_p) for k in ("head", "tail", "ring_packet", "ring_len", "ring_payload_len", "ring_dst")]


class sg_routing_view(C.Structure):
    _fields_ = [("n", C.c_uint32), ("node_ids", C.c_void_p), ("cells", C.c_void_p), ("n_wide", C.c_uint64),
                ("pinned", C.c_uint32)]


class sg_round(C.Structure):
    _fields_ = [("round_end_ns", C.c_uint64), ("sim_end_ns", C.c_uint64), ("bootstrap_end_ns", C.c_uint64)]


class sg_packets(C.Structure):
    _fields_ = [("n_packets", C.c_uint32), ("src_host", C.c_void_p), ("dst_ipv4", C.c_void_p),
                ("payload_len", C.c_void_p), ("send_time_ns", C.c_void_p), ("rng_skip", C.c_void_p)]


class sg_deliveries(C.Structure):
    _fields_ = [("status", C.c_void_p), ("deliver_time_ns", C.c_void_p), ("event_id", C.c_void_p),
                ("dst_order", C.c_void_p), ("dst_offsets", C.c_void_p)]


class sg_round_stats(C.Structure):
    _fields_ = [("n_delivered", C.c_uint64), ("min_deliver_time_ns", C.c_uint64),
                ("min_used_latency_ns", C.c_uint64)]


_lib = None
_lib_version = None


def abi_version() -> int:
    """The loaded library's ABI version (older ones only via SHADOW_GPU_LIB, for A/B tools)."""
    load()
    return _lib_version


def require_abi(v: int, what: str) -> None:
    """Raise if the loaded library predates ABI `v`, which `what` needs (its structs differ)."""
    if abi_version() < v:
        raise ShadowGpuUnavailable(f"{what} needs ABI {v}; the loaded library is ABI {_lib_version}")


def load(path: str | None = None):
    """Load libshadow_gpu.so; raises ShadowGpuUnavailable (never falls back)."""
    global _lib, _lib_version
    if _lib is not None:
        return _lib
    path = path or os.environ.get("SHADOW_GPU_LIB", LIB_PATH)
    # One HIP runtime per process: torch bundles its own libamdhip64.so (soname
    # libamdhip64.so.7).  If our library loaded first, /opt/rocm's runtime would
    # come in too and whichever initialised second would see no device.  Loading
    # torch first lets our NEEDED libamdhip64.so.7 resolve to the loaded copy.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(path):
        raise ShadowGpuUnavailable(
            f"{path} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(hipcc --offload-arch=gfx950); there is no CPU fallback")
    try:
        L = C.CDLL(path)
    except OSError as e:
        raise ShadowGpuUnavailable(f"cannot load {path}: {e}") from e
    vp, u32, u64, i32 = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int32
    u32p, u64p = C.POINTER(C.c_uint32), C.POINTER(C.c_uint64)
    sig = {
        "sg_abi_version": (i32, []),
        "sg_ctx_create": (i32, [i32, C.POINTER(vp)]),
        "sg_ctx_destroy": (None, [vp]),
        "sg_ctx_set_stream": (i32, [vp, vp]),
        "sg_ctx_stream": (vp, [vp]),
        "sg_ctx_synchronize": (i32, [vp]),
        "sg_ctx_last_error": (C.c_char_p, [vp]),
        "sg_ctx_last_error_pair": (None, [vp, u32p, u32p]),
        "sg_ctx_enable_timers": (i32, [vp, i32]),
        "sg_ctx_read_timer": (i32, [vp, C.c_char_p, C.POINTER(C.c_double), u64p, C.POINTER(C.c_double)]),
        "sg_gml_parse": (i32, [C.c_char_p, C.c_size_t, C.POINTER(vp), C.c_char_p, C.c_size_t]),
        "sg_gml_parse_threads": (i32, [C.c_char_p, C.c_size_t, u32, C.POINTER(vp), C.c_char_p, C.c_size_t]),
        "sg_gml_load": (i32, [C.c_char_p, u32, u32, C.POINTER(vp), C.c_char_p, C.c_size_t]),
        "sg_gml_graph": (i32, [vp, C.POINTER(sg_graph)]),
        "sg_gml_node_index": (i32, [vp, u32, u32p]),
        "sg_gml_destroy": (None, [vp]),
        "sg_net_create": (i32, [vp, C.POINTER(sg_graph), C.POINTER(vp)]),
        "sg_net_destroy": (None, [vp]),
        "sg_routing_build": (i32, [vp, vp, vp, u32, u32, u32, u32, vp, vp]),
        "sg_routing_min_latency": (i32, [vp, vp, C.c_size_t, u64p]),
        "sg_routing_info_create": (i32, [u32, vp, C.POINTER(vp)]),
        "sg_routing_info_destroy": (None, [vp]),
        "sg_routing_info_fill": (i32, [vp, vp, vp, u32, vp]),
        "sg_routing_info_set_rows": (i32, [vp, u32, u32, vp, vp]),
        "sg_routing_info_view": (i32, [vp, C.POINTER(sg_routing_view)]),
        "sg_routing_info_rows": (i32, [vp, u32, u32, vp, vp]),
        "sg_routing_info_index": (i32, [vp, u32, C.POINTER(C.c_uint32)]),
        "sg_routing_info_path": (i32, [vp, u32, u32, u64p, C.POINTER(C.c_float)]),
        "sg_routing_info_smallest_latency": (i32, [vp, u64p]),
        "sg_routing_info_increment_packet_count": (i32, [vp, u32, u32]),
        "sg_routing_info_packet_count": (u64, [vp, u32, u32]),
        "sg_routing_info_set_addresses": (i32, [vp, u32, vp, vp]),
        "sg_worker_get_latency": (i32, [vp, u32, u32, u64p]),
        "sg_worker_get_reliability": (i32, [vp, u32, u32, C.POINTER(C.c_float)]),
        "sg_worker_is_routable": (i32, [vp, u32, u32]),
        "sg_hosts_create": (i32, [vp, u32, vp, vp, vp, C.POINTER(vp)]),
        "sg_hosts_get_state": (i32, [vp, vp, vp]),
        "sg_hosts_set_state": (i32, [vp, vp, vp]),
        "sg_hosts_skip": (i32, [vp, u32, vp, vp]),
        "sg_hosts_destroy": (None, [vp]),
        "sg_deliver_round": (i32, [vp, vp, C.POINTER(sg_table), C.POINTER(sg_round), C.POINTER(sg_packets),
                                   C.POINTER(sg_deliveries), C.POINTER(sg_round_stats)]),
        "sg_deliver_source": (i32, [vp, vp, C.POINTER(sg_table), C.POINTER(sg_round), C.POINTER(sg_packets),
                                    vp, vp, vp, vp, u32, vp, u32p, C.POINTER(sg_round_stats)]),
        "sg_deliver_bucket": (i32, [vp, vp, u32, vp, u32, u32, vp, vp]),
        "sg_deliver_source_padded": (i32, [vp, vp, C.POINTER(sg_table), C.POINTER(sg_round), C.POINTER(sg_packets),
                                           vp, vp, vp, vp, u32, u32, vp, vp, vp]),
        "sg_deliver_bucket_padded": (i32, [vp, vp, u32, u32, vp, u32, vp, u32, u32, vp, vp,
                                           C.POINTER(sg_round_stats), vp, C.POINTER(C.c_uint32)]),
        "sg_deliver_pad_to_compact": (i32, [vp, vp, u32, u32, vp, vp]),
        "sg_table_pack": (i32, [vp, C.POINTER(sg_table), vp, u32p]),
        "sg_codel_create": (i32, [vp, u32, u32, C.POINTER(vp)]),
        "sg_codel_destroy": (None, [vp]),
        "sg_codel_run": (i32, [vp, vp, C.POINTER(sg_codel_events), vp, vp, u32, u64p]),
        "sg_codel_ring_cap": (u32, [vp]),
        "sg_codel_get_state": (i32, [vp, C.POINTER(sg_codel_state)]),
        "sg_codel_set_state": (i32, [vp, C.POINTER(sg_codel_state)]),
        "sg_inbound_create": (i32, [vp, u32, vp, u32, C.POINTER(vp)]),
        "sg_inbound_destroy": (None, [vp]),
        "sg_inbound_ring_cap": (u32, [vp]),
        "sg_inbound_run": (i32, [vp, vp, C.POINTER(sg_inbound_arrivals), u64, u64, u64, vp, vp, vp, u32, u64p]),
        "sg_inbound_run_ordered": (i32, [vp, vp, C.POINTER(sg_inbound_arrivals), u64, u64, u64, vp, vp, vp, u32, vp,
                                         vp, u64p]),
        "sg_ctx_set_packet_counters": (i32, [vp, vp, u64]),
        "sg_inbound_get_state": (i32, [vp, C.POINTER(sg_codel_state), C.POINTER(sg_inbound_relay_state)]),
        "sg_hosts_event_ctr": (vp, [vp]),
        "sg_outbound_create": (i32, [vp, u32, vp, vp, u32, C.POINTER(vp)]),
        "sg_outbound_destroy": (None, [vp]),
        "sg_outbound_ring_cap": (u32, [vp]),
        "sg_outbound_run": (i32, [vp, vp, C.POINTER(sg_outbound_sends), u64, u64, u64, vp, vp, vp, u32,
                                  C.POINTER(sg_outbound_sent), C.POINTER(C.c_uint32)]),
        "sg_outbound_get_state": (i32, [vp, C.POINTER(sg_outbound_queue_state), C.POINTER(sg_inbound_relay_state)]),
        "sg_comm_unique_id": (i32, [vp]),
        "sg_comm_create": (i32, [vp, vp, u32, u32, C.POINTER(vp)]),
        "sg_comm_destroy": (None, [vp]),
        "sg_comm_allgather_rows": (i32, [vp, vp, vp, u32, u32]),
        "sg_comm_exchange_padded": (i32, [vp, vp, vp, u32, vp, vp]),
        "sg_comm_alltoallv_records": (i32, [vp, vp, u32p, vp, u32p]),
        "sg_comm_allgather_u64": (i32, [vp, vp, vp, u32]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name, None)
        if f is None:  # only an older library given via SHADOW_GPU_LIB (A/B tools) lacks symbols
            continue
        f.restype = res
        f.argtypes = args
    v = L.sg_abi_version()
    # An older library given via SHADOW_GPU_LIB (A/B tools: routing builds only) is
    # accepted, and its version recorded: the calls whose structs changed since check
    # it with require_abi (v5: routing view cells, packets' rng_skip; v6: outbound
    # send keys and relay task ids) instead of misreading memory.
    if v != SG_ABI_VERSION and not (path != LIB_PATH and 1 <= v < SG_ABI_VERSION):
        raise ShadowGpuUnavailable(f"ABI version mismatch: library {v}, bindings {SG_ABI_VERSION}")
    _lib = L
    _lib_version = int(v)
    return L


def check(ctx_handle, rc: int) -> None:
    if rc == SG_OK:
        return
    L = load()
    msg = L.sg_ctx_last_error(ctx_handle).decode(errors="replace") if ctx_handle else f"status {rc}"
    r, c = C.c_uint32(), C.c_uint32()
    if ctx_handle:
        L.sg_ctx_last_error_pair(ctx_handle, C.byref(r), C.byref(c))
    raise ShadowGpuError(rc, msg, (r.value, c.value))
