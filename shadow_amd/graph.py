"""Host-side mirror of Shadow's network-graph interface over the HIP core.

Names, argument meaning and errors follow src/main/network/graph/mod.rs and
src/main/core/sim_config.rs so that a test written against the reference reads
the same here:

    graph = NetworkGraph.parse(gml_text)                       # graph/mod.rs:134
    n0 = graph.node_id_to_index(0)                             # graph/mod.rs:126
    paths = graph.compute_shortest_paths([n0, n1, n2])         # graph/mod.rs:183
    paths[(n0, n1)].latency_ns
    routing = generate_routing_info(graph, {0, 1, 2}, True)    # sim_config.rs:411
    routing.path(0, 1)                                         # graph/mod.rs:448

All computation runs in libshadow_gpu.so on the GPU; there is no CPU path.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Dict, Iterable, Iterator, List, Optional, Sequence, Tuple

import numpy as np

from . import _capi
from ._capi import ShadowGpuError, check, load


# ---------------------------------------------------------------------------
# Context
# ---------------------------------------------------------------------------
class Context:
    """One GPU (HIP device) + stream + workspace (sg_ctx)."""

    def __init__(self, device: int = 0, stream: Optional[int] = None):
        L = load()
        h = C.c_void_p()
        rc = L.sg_ctx_create(int(device), C.byref(h))
        if rc != _capi.SG_OK:
            why = (L.sg_ctx_last_error(None) or b"").decode(errors="replace")
            raise ShadowGpuError(rc, f"sg_ctx_create(device={device}) failed with status {rc}: {why}")
        self.handle = h
        self.device = int(device)
        if stream is not None:
            self.set_stream(stream)

    def set_stream(self, stream: Optional[int]) -> None:
        """Launch on `stream` (a hipStream_t as int, e.g. torch's cuda_stream); None = own stream."""
        check(self.handle, load().sg_ctx_set_stream(self.handle, C.c_void_p(stream or 0)))

    @property
    def stream(self) -> int:
        return load().sg_ctx_stream(self.handle) or 0

    def synchronize(self) -> None:
        check(self.handle, load().sg_ctx_synchronize(self.handle))

    def set_packet_counters(self, counts=None) -> None:
        """RoutingInfo::increment_packet_count on the device (sg_ctx_set_packet_counters): a
        zeroed int64 device tensor with a cell per routing-table cell; every delivered packet of
        this context's later rounds adds one at its path's cell.  None turns counting off."""
        if counts is None:
            check(self.handle, load().sg_ctx_set_packet_counters(self.handle, None, 0))
            return
        if counts.dtype.itemsize != 8 or not counts.is_cuda or not counts.is_contiguous():
            raise ValueError("packet counters: a contiguous 8-byte device tensor")
        self._packet_counts = counts  # kept alive while the library holds the pointer
        check(self.handle, load().sg_ctx_set_packet_counters(self.handle, counts.data_ptr(), counts.numel()))

    def enable_timers(self, enable: bool = True, count_work: bool = False) -> None:
        """Per-kernel HIP-event timers on this context's stream (resets them).

        count_work: run the counting variants of data-dependent kernels (the
        relaxation kernel's lane-relaxation count); time them in a separate run.
        """
        mode = (1 | (2 if count_work else 0)) if enable else 0
        check(self.handle, load().sg_ctx_enable_timers(self.handle, mode))

    def read_timer(self, kernel: str):
        """(total device ms, launches, declared algorithmic work) for one kernel."""
        t, n, w = C.c_double(), C.c_uint64(), C.c_double()
        check(self.handle, load().sg_ctx_read_timer(self.handle, kernel.encode(), C.byref(t), C.byref(n), C.byref(w)))
        return t.value, n.value, w.value

    def close(self) -> None:
        if getattr(self, "handle", None):
            load().sg_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_default_ctx: Dict[int, Context] = {}


def default_context(device: int = 0) -> Context:
    if device not in _default_ctx:
        _default_ctx[device] = Context(device)
    return _default_ctx[device]


# ---------------------------------------------------------------------------
# PathProperties (graph/mod.rs:297-340)
# ---------------------------------------------------------------------------
@dataclass(frozen=True)
class PathProperties:
    latency_ns: int
    packet_loss: np.float32

    def _key(self):
        return (self.latency_ns, float(self.packet_loss))

    # graph/mod.rs:305-320: latency first, then packet loss
    def __lt__(self, other):
        return self._key() < other._key()

    def __le__(self, other):
        return self._key() <= other._key()

    def __eq__(self, other):
        return isinstance(other, PathProperties) and self._key() == other._key()

    def __hash__(self):
        return hash(self._key())

    # graph/mod.rs:322-331 (f32 ops, one rounding each)
    def __add__(self, other: "PathProperties") -> "PathProperties":
        one = np.float32(1.0)
        a, b = np.float32(self.packet_loss), np.float32(other.packet_loss)
        return PathProperties(self.latency_ns + other.latency_ns,
                              np.float32(one - np.float32(np.float32(one - a) * np.float32(one - b))))


DEFAULT_PATH = PathProperties(0, np.float32(0.0))


class PathTable:
    """Dense result of compute_shortest_paths / get_direct_paths.

    Behaves like the reference's HashMap<(NodeIndex, NodeIndex), PathProperties>
    (graph/mod.rs:186): keys are (src, dst) node indices from `nodes`; the
    arrays `latency_ns` (u64) and `packet_loss` (f32) are [n_used x n_used]
    with row = source in `nodes` order.
    """

    def __init__(self, nodes: Sequence[int], latency_ns: np.ndarray, packet_loss: np.ndarray):
        self.nodes = [int(x) for x in nodes]
        self.index = {n: i for i, n in enumerate(self.nodes)}
        self.latency_ns = latency_ns
        self.packet_loss = packet_loss

    def __len__(self) -> int:
        return len(self.nodes) ** 2

    def get(self, key: Tuple[int, int]) -> Optional[PathProperties]:
        i, j = self.index.get(key[0]), self.index.get(key[1])
        if i is None or j is None:
            return None
        return PathProperties(int(self.latency_ns[i, j]), np.float32(self.packet_loss[i, j]))

    def __getitem__(self, key: Tuple[int, int]) -> PathProperties:
        p = self.get(key)
        if p is None:
            raise KeyError(key)
        return p

    def __contains__(self, key) -> bool:
        return key[0] in self.index and key[1] in self.index

    def keys(self) -> Iterator[Tuple[int, int]]:
        for a in self.nodes:
            for b in self.nodes:
                yield (a, b)

    def items(self):
        for k in self.keys():
            yield k, self[k]


# ---------------------------------------------------------------------------
# NetworkGraph (graph/mod.rs:113-294)
# ---------------------------------------------------------------------------
class NetworkGraph:
    def __init__(self, n_nodes: int, edge_src, edge_dst, edge_latency_ns, edge_packet_loss,
                 directed: bool, node_ids: Optional[Sequence[int]] = None, ctx: Optional[Context] = None):
        self._ctx = ctx
        self.n_nodes = int(n_nodes)
        self.directed = bool(directed)
        self.edge_src = np.ascontiguousarray(edge_src, dtype=np.uint32)
        self.edge_dst = np.ascontiguousarray(edge_dst, dtype=np.uint32)
        self.edge_latency_ns = np.ascontiguousarray(edge_latency_ns, dtype=np.uint64)
        self.edge_packet_loss = np.ascontiguousarray(edge_packet_loss, dtype=np.float32)
        # GML node ids; None: each node's index (built only if asked for, and not passed to
        # sg_net_create, which then names nodes by index -- a one-shot build skips both)
        self._node_ids = None if node_ids is None else np.ascontiguousarray(node_ids, dtype=np.uint32)
        self._id_to_index = None  # built on first lookup
        self._net = None

    @property
    def node_ids(self) -> np.ndarray:
        """The GML node id of each node index."""
        if self._node_ids is None:
            self._node_ids = np.arange(self.n_nodes, dtype=np.uint32)
        return self._node_ids

    @property
    def ctx(self) -> Context:
        if self._ctx is None:
            self._ctx = default_context()
        return self._ctx

    def _graph_struct(self) -> _capi.sg_graph:
        g = _capi.sg_graph()
        g.n_nodes = self.n_nodes
        g.n_edges = len(self.edge_src)
        # (the arrays' addresses straight from the array interface: ndarray.ctypes builds a helper
        # object per call, and this runs in every one-shot build)
        ptr = lambda a, t: C.cast(a.__array_interface__["data"][0], C.POINTER(t))
        g.edge_src = ptr(self.edge_src, C.c_uint32)
        g.edge_dst = ptr(self.edge_dst, C.c_uint32)
        g.edge_latency_ns = ptr(self.edge_latency_ns, C.c_uint64)
        g.edge_packet_loss = ptr(self.edge_packet_loss, C.c_float)
        g.node_gml_id = None if self._node_ids is None else ptr(self._node_ids, C.c_uint32)
        g.directed = 1 if self.directed else 0
        return g

    def _ensure_net(self):
        """Upload the edge list once (sg_net_create) on first use of the device."""
        if self._net is None:
            self._upload()
        return self._net

    def _upload(self) -> None:
        L = load()
        g = self._graph_struct()
        h = C.c_void_p()
        check(self.ctx.handle, L.sg_net_create(self.ctx.handle, C.byref(g), C.byref(h)))
        self._net = h

    def close(self) -> None:
        """Release the device graph (sg_net_destroy) now rather than at garbage collection."""
        if self._net:
            load().sg_net_destroy(self._net)
            self._net = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @classmethod
    def parse(cls, graph_text, ctx: Optional[Context] = None, threads: int = 0) -> "NetworkGraph":
        """NetworkGraph::parse (graph/mod.rs:134-181); raises ShadowGpuError(SG_ERR_PARSE).
        graph_text: str or bytes (UTF-8).  threads: host threads for the parse (0 = min(cores, 16))."""
        L = load()
        raw = graph_text.encode() if isinstance(graph_text, str) else bytes(graph_text)
        h = C.c_void_p()
        err = C.create_string_buffer(512)
        rc = L.sg_gml_parse_threads(raw, len(raw), int(threads), C.byref(h), err, len(err))
        if rc != _capi.SG_OK:
            raise ShadowGpuError(rc, err.value.decode(errors="replace") or f"parse status {rc}")
        return cls._from_handle(h, ctx)

    @classmethod
    def _from_handle(cls, h, ctx) -> "NetworkGraph":
        L = load()
        try:
            g = _capi.sg_graph()
            check(None, L.sg_gml_graph(h, C.byref(g)))
            n, m = g.n_nodes, g.n_edges
            arr = lambda p, cnt, dt: np.ctypeslib.as_array(p, shape=(cnt,)).astype(dt) if cnt else np.zeros(0, dt)
            return cls(n, arr(g.edge_src, m, np.uint32), arr(g.edge_dst, m, np.uint32),
                       arr(g.edge_latency_ns, m, np.uint64), arr(g.edge_packet_loss, m, np.float32),
                       bool(g.directed), arr(g.node_gml_id, n, np.uint32), ctx)
        finally:
            L.sg_gml_destroy(h)

    @classmethod
    def from_file(cls, path, compression: Optional[str] = None, ctx: Optional[Context] = None,
                  threads: int = 0) -> "NetworkGraph":
        """load_network_graph + NetworkGraph::parse (graph/mod.rs:483-513) in the native
        library (sg_gml_load): a GML file, plain or xz-compressed (compression="xz", read_xz
        :484-496; decompressed by the system liblzma), checked to be UTF-8
        (String::from_utf8), then parsed on `threads` threads."""
        if compression not in (None, "xz"):
            raise ValueError(f"unknown compression {compression!r} (configuration.rs:985-988: xz)")
        L = load()
        h = C.c_void_p()
        err = C.create_string_buffer(512)
        rc = L.sg_gml_load(str(path).encode(), 1 if compression == "xz" else 0, int(threads), C.byref(h), err,
                           len(err))
        if rc != _capi.SG_OK:
            raise ShadowGpuError(rc, err.value.decode(errors="replace") or f"load status {rc}")
        return cls._from_handle(h, ctx)

    def node_id_to_index(self, node_id: int) -> Optional[int]:
        if self._id_to_index is None:  # graph/mod.rs:155-162: a later duplicate id wins
            self._id_to_index = {int(i): k for k, i in enumerate(self.node_ids)}
        return self._id_to_index.get(int(node_id))

    def node_index_to_id(self, index: int) -> Optional[int]:
        return int(self.node_ids[index]) if 0 <= index < self.n_nodes else None

    # -- routing ------------------------------------------------------------
    def _build(self, nodes: Sequence[int], shortest: bool) -> PathTable:
        L = load()
        used = np.ascontiguousarray(nodes, dtype=np.uint32)
        nu = len(used)
        lat = np.zeros((nu, nu), np.uint64)
        loss = np.zeros((nu, nu), np.float32)
        flags = _capi.SG_ROUTE_SHORTEST_PATH if shortest else 0
        check(self.ctx.handle, L.sg_routing_build(self.ctx.handle, self._ensure_net(), used.ctypes.data, nu, 0, nu, flags,
                                                  lat.ctypes.data, loss.ctypes.data))
        return PathTable(used.tolist(), lat, loss)

    def compute_shortest_paths(self, nodes: Sequence[int]) -> PathTable:
        """graph/mod.rs:183-228 (bit-exact latency and f32 loss)."""
        return self._build(nodes, True)

    def get_direct_paths(self, nodes: Sequence[int]) -> PathTable:
        """graph/mod.rs:230-252."""
        return self._build(nodes, False)

    def build_rows_device(self, nodes: Sequence[int], row_begin: int, row_end: int, out_latency_ptr: int,
                          out_loss_ptr: int, shortest: bool = True) -> None:
        """Rows [row_begin, row_end) into caller-owned device buffers (sharded build)."""
        L = load()
        used = np.ascontiguousarray(nodes, dtype=np.uint32)
        flags = (_capi.SG_ROUTE_SHORTEST_PATH if shortest else 0) | _capi.SG_ROUTE_OUT_DEVICE
        check(self.ctx.handle, L.sg_routing_build(self.ctx.handle, self._ensure_net(), used.ctypes.data, len(used),
                                                  int(row_begin), int(row_end), flags, C.c_void_p(out_latency_ptr),
                                                  C.c_void_p(out_loss_ptr)))

    def min_latency_device(self, latency_ptr: int, count: int) -> int:
        out = C.c_uint64()
        check(self.ctx.handle, load().sg_routing_min_latency(self.ctx.handle, C.c_void_p(latency_ptr), count,
                                                             C.byref(out)))
        return out.value


# ---------------------------------------------------------------------------
# RoutingInfo (graph/mod.rs:432-481) keyed by GML node id: a dense host table
# owned by libshadow_gpu (sg_routing_info, sg_route_info.hip)
# ---------------------------------------------------------------------------
class RoutingInfo:
    """RoutingInfo<u32>: path(start, end), get_smallest_latency_ns and the packet
    counters, over a dense table of 8-byte (latency, loss) cells in pinned host
    memory (row = source, in `node_ids` order).  `latency_ns` / `packet_loss` /
    `rows()` decode copies; `cells` is the zero-copy packed view.  With addresses attached
    (set_addresses) it also answers WorkerShared::latency / reliability /
    is_routable (worker.rs:517-555)."""

    def __init__(self, node_ids: Sequence[int], latency_ns: Optional[np.ndarray] = None,
                 packet_loss: Optional[np.ndarray] = None):
        L = load()
        ids = np.ascontiguousarray(node_ids, dtype=np.uint32)
        h = C.c_void_p()
        rc = L.sg_routing_info_create(len(ids), ids.ctypes.data, C.byref(h))
        if rc != _capi.SG_OK:
            raise ShadowGpuError(rc, "sg_routing_info_create failed (duplicate node id?)")
        self.handle = h
        self.node_ids = [int(x) for x in ids]
        self.n = len(ids)
        if latency_ns is not None:
            self.set_rows(0, np.asarray(latency_ns, np.uint64), np.asarray(packet_loss, np.float32))

    def __del__(self):
        h = getattr(self, "handle", None)
        if h:
            load().sg_routing_info_destroy(h)
            self.handle = None

    def fill(self, graph: "NetworkGraph", nodes: Sequence[int], use_shortest_paths: bool = True) -> None:
        """sg_routing_info_fill: the whole table from the GPU (nodes = petgraph indices of node_ids)."""
        idx = np.ascontiguousarray(nodes, dtype=np.uint32)
        assert len(idx) == self.n
        flags = _capi.SG_ROUTE_SHORTEST_PATH if use_shortest_paths else 0
        check(graph.ctx.handle, load().sg_routing_info_fill(graph.ctx.handle, graph._ensure_net(), idx.ctypes.data,
                                                             flags, self.handle))

    def set_rows(self, row_begin: int, latency_ns: np.ndarray, packet_loss: np.ndarray) -> None:
        lat = np.ascontiguousarray(latency_ns, np.uint64).reshape(-1, self.n)
        loss = np.ascontiguousarray(packet_loss, np.float32).reshape(-1, self.n)
        rc = load().sg_routing_info_set_rows(self.handle, int(row_begin), int(row_begin) + lat.shape[0],
                                             lat.ctypes.data, loss.ctypes.data)
        if rc != _capi.SG_OK:
            raise ShadowGpuError(rc, "sg_routing_info_set_rows: bad row range")

    def _view(self):
        v = _capi.sg_routing_view()
        load().sg_routing_info_view(self.handle, C.byref(v))
        return v

    def rows(self, row_begin: int = 0, row_end: Optional[int] = None):
        """Rows [row_begin, row_end) decoded from the 8-byte cells (sg_routing_info_rows): a
        (latency u64, loss f32) pair of new arrays."""
        _capi.require_abi(5, "RoutingInfo.rows")
        row_end = self.n if row_end is None else int(row_end)
        k = max(0, row_end - int(row_begin))
        lat = np.empty((k, self.n), np.uint64)
        loss = np.empty((k, self.n), np.float32)
        rc = load().sg_routing_info_rows(self.handle, int(row_begin), row_end, lat.ctypes.data, loss.ctypes.data)
        if rc != _capi.SG_OK:
            raise ShadowGpuError(rc, "sg_routing_info_rows: bad row range")
        return lat, loss

    @property
    def latency_ns(self) -> np.ndarray:
        """[n x n] latencies (a copy, decoded from the cells)."""
        return self.rows()[0]

    @property
    def packet_loss(self) -> np.ndarray:
        """[n x n] losses (a copy)."""
        return self.rows()[1]

    @property
    def cells(self) -> np.ndarray:
        """Zero-copy [n x n] view of the packed cells (latency << 32 | bits(loss); SG_CELL_WIDE in the
        upper half for paths of 2^32 - 1 ns or more).  The array keeps this object alive."""
        _capi.require_abi(5, "RoutingInfo.cells")
        v = self._view()
        if not self.n:
            return np.zeros((0, 0), np.uint64)
        buf = (C.c_uint64 * (self.n * self.n)).from_address(v.cells)
        buf._owner = self  # the frombuffer base chain keeps the table alive
        return np.frombuffer(buf, dtype=np.uint64).reshape(self.n, self.n)

    @property
    def pinned(self) -> bool:
        return bool(self._view().pinned)

    def index(self, node_id: int) -> Optional[int]:
        r = C.c_uint32()
        return int(r.value) if load().sg_routing_info_index(self.handle, int(node_id), C.byref(r)) == 0 else None

    def path(self, start: int, end: int) -> Optional[PathProperties]:
        """graph/mod.rs:448-450."""
        lat, loss = C.c_uint64(), C.c_float()
        if not load().sg_routing_info_path(self.handle, int(start), int(end), C.byref(lat), C.byref(loss)):
            return None
        return PathProperties(int(lat.value), np.float32(loss.value))

    def increment_packet_count(self, start: int, end: int) -> None:
        """graph/mod.rs:453-460 (saturating; the reference's caller unwraps an unknown pair)."""
        rc = load().sg_routing_info_increment_packet_count(self.handle, int(start), int(end))
        if rc != _capi.SG_OK:
            raise KeyError((start, end))

    def packet_count(self, start: int, end: int) -> int:
        return int(load().sg_routing_info_packet_count(self.handle, int(start), int(end)))

    def get_smallest_latency_ns(self) -> Optional[int]:
        """graph/mod.rs:478-480: min over every entry, self pairs included."""
        out = C.c_uint64()
        return int(out.value) if load().sg_routing_info_smallest_latency(self.handle, C.byref(out)) else None

    # -- WorkerShared lookups (worker.rs:517-555), addresses as host-order u32 ----
    def set_addresses(self, ipv4: Sequence[int], node_ids: Sequence[int]) -> None:
        ips = np.ascontiguousarray(ipv4, np.uint32)
        ids = np.ascontiguousarray(node_ids, np.uint32)
        rc = load().sg_routing_info_set_addresses(self.handle, len(ips), ips.ctypes.data, ids.ctypes.data)
        if rc != _capi.SG_OK:
            raise ShadowGpuError(rc, "IP address has already been assigned")

    @staticmethod
    def _be(ip: int) -> int:
        return int.from_bytes(int(ip).to_bytes(4, "big"), "little")  # in_addr_t: network byte order

    def latency(self, src_ip: int, dst_ip: int) -> Optional[int]:
        out = C.c_uint64()
        rc = load().sg_worker_get_latency(self.handle, self._be(src_ip), self._be(dst_ip), C.byref(out))
        return int(out.value) if rc == _capi.SG_OK else None

    def reliability(self, src_ip: int, dst_ip: int) -> Optional[np.float32]:
        out = C.c_float()
        rc = load().sg_worker_get_reliability(self.handle, self._be(src_ip), self._be(dst_ip), C.byref(out))
        return np.float32(out.value) if rc == _capi.SG_OK else None

    def is_routable(self, src_ip: int, dst_ip: int) -> bool:
        return bool(load().sg_worker_is_routable(self.handle, self._be(src_ip), self._be(dst_ip)))


def generate_routing_info(graph: NetworkGraph, node_ids: Iterable[int], use_shortest_paths: bool) -> RoutingInfo:
    """sim_config.rs:411-448: used GML ids -> petgraph indices, build straight into
    the dense host RoutingInfo keyed by the ids (no HashMap, no remap pass)."""
    ids = list(node_ids)
    idx = []
    for x in ids:
        i = graph.node_id_to_index(x)
        if i is None:
            raise KeyError(f"node id {x} not in graph")
        idx.append(i)
    # an id that maps to an index twice collapses in the reference's HashMap; ids are unique here
    ri = RoutingInfo([graph.node_index_to_id(i) for i in idx])
    try:
        ri.fill(graph, idx, use_shortest_paths)
    except ShadowGpuError as e:
        what = "shortest paths" if use_shortest_paths else "the direct paths"
        raise ShadowGpuError(e.code, f"Failed to compute {what} between graph nodes: {e}", e.pair) from None
    return ri


# ---------------------------------------------------------------------------
# IpAssignment (graph/mod.rs:352-430)
# ---------------------------------------------------------------------------
def ipv4_to_u32(s: str) -> int:
    a, b, c, d = (int(x) for x in s.split("."))
    return (a << 24) | (b << 16) | (c << 8) | d


def u32_to_ipv4(x: int) -> str:
    return f"{(x >> 24) & 255}.{(x >> 16) & 255}.{(x >> 8) & 255}.{x & 255}"


class IpAssignment:
    def __init__(self):
        self.map: Dict[int, int] = {}
        self.last_assigned_addr = ipv4_to_u32("11.0.0.0")

    @staticmethod
    def increment_address(addr: int) -> int:
        inc = 1
        while True:
            nxt = (addr + inc) & 0xFFFFFFFF
            if (nxt & 0xFF) in (0, 255):  # skip .0 and .255 (graph/mod.rs:414-417)
                inc += 1
                continue
            return nxt

    def assign(self, node_id: int) -> int:
        while True:
            ip = self.increment_address(self.last_assigned_addr)
            self.last_assigned_addr = ip
            if ip not in self.map:
                self.map[ip] = node_id
                return ip

    def assign_ip(self, node_id: int, ip: int) -> None:
        if ip in self.map:
            raise ShadowGpuError(_capi.SG_ERR_DUPLICATE_IP, "IP address has already been assigned")
        self.map[ip] = node_id

    def get_node(self, ip: int) -> Optional[int]:
        return self.map.get(ip)

    def get_nodes(self) -> set:
        return set(self.map.values())
