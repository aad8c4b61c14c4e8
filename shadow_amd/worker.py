"""Round-batched packet delivery: host-side mirror of Worker::send_packet.

The reference calls Worker::send_packet once per packet from N worker threads
(src/main/core/worker.rs:322-397) and pushes each delivered packet into the
destination's locked EventQueue (worker.rs:597-607).  Here a round's sends are
logged as a device SoA (`PacketBatch`) and `deliver_round` runs the whole
round on the GPU at the round boundary (exact: see sg_deliver.hip).

Device memory is allocated through torch (plumbing only); every computation is
a HIP kernel in libshadow_gpu.so.
"""
from __future__ import annotations

import ctypes as C
import weakref
from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import _capi
from ._capi import check, load
from .graph import Context, default_context


def _torch():
    import torch  # plumbing for device memory / streams

    return torch


def _key(obj, fields):
    return tuple(id(getattr(obj, f)) for f in fields)


class _Versioned:
    """Counts assignments to the tensor fields a ctypes struct is built from (_FIELDS), so a
    cached call can check in one comparison that none was replaced."""
    _FIELDS = ()

    def __setattr__(self, name, value):
        if name in self._FIELDS:
            object.__setattr__(self, "_ver", self.__dict__.get("_ver", 0) + 1)
        object.__setattr__(self, name, value)

    def c_struct_key(self):
        return self.__dict__.get("_ver", 0)


def _cached(obj, fields, build):
    """ctypes struct for obj, rebuilt only when one of its tensor fields is replaced
    (a round loop reuses the same buffers: no per-round data_ptr() / struct setup)."""
    key = _key(obj, fields)
    c = obj.__dict__.get("_c")
    if c is None or c[0] != key:
        c = (key, build())
        obj.__dict__["_c"] = c
    return c[1]


def _dev_u32(x, device):
    torch = _torch()
    if isinstance(x, torch.Tensor):
        assert x.dtype == torch.int32 and x.is_cuda and x.is_contiguous()
        return x
    return torch.from_numpy(np.ascontiguousarray(x, dtype=np.uint32).view(np.int32)).to(device)


def _dev_u64(x, device):
    torch = _torch()
    if isinstance(x, torch.Tensor):
        assert x.dtype == torch.int64 and x.is_cuda and x.is_contiguous()
        return x
    return torch.from_numpy(np.ascontiguousarray(x, dtype=np.uint64).view(np.int64)).to(device)


class HostTable:
    """sg_hosts: per-host address, routing index, Xoshiro256++ stream, event-id counter.

    host_seed[h] = HostInfo.seed (sim_config.rs:221-242); the stream is
    Xoshiro256PlusPlus::seed_from_u64(seed) (host.rs:221).
    """

    def __init__(self, host_ipv4, host_route_idx, host_seed, ctx: Optional[Context] = None):
        self.ctx = ctx or default_context()
        ip = np.ascontiguousarray(host_ipv4, dtype=np.uint32)
        route = np.ascontiguousarray(host_route_idx, dtype=np.uint32)
        seed = np.ascontiguousarray(host_seed, dtype=np.uint64)
        assert len(ip) == len(route) == len(seed)
        self.n = len(ip)
        self.host_ipv4, self.host_route_idx = ip, route
        h = C.c_void_p()
        check(self.ctx.handle, load().sg_hosts_create(self.ctx.handle, self.n, ip.ctypes.data, route.ctypes.data,
                                                      seed.ctypes.data, C.byref(h)))
        self.handle = h

    def get_state(self):
        rng = np.zeros((self.n, 4), np.uint64)
        ctr = np.zeros(self.n, np.uint64)
        check(self.ctx.handle, load().sg_hosts_get_state(self.handle, rng.ctypes.data, ctr.ctypes.data))
        return rng, ctr

    def set_state(self, rng: Optional[np.ndarray] = None, ctr: Optional[np.ndarray] = None) -> None:
        r = None if rng is None else np.ascontiguousarray(rng, dtype=np.uint64)
        c = None if ctr is None else np.ascontiguousarray(ctr, dtype=np.uint64)
        check(self.ctx.handle, load().sg_hosts_set_state(self.handle, None if r is None else r.ctypes.data,
                                                         None if c is None else c.ctypes.data))

    def skip(self, host_ids, steps) -> None:
        """Advance hosts' device RNG streams by the steps other consumers took
        (sg_hosts_skip; see PacketBatch.rng_skip).  A host may repeat."""
        ids = np.ascontiguousarray(host_ids, dtype=np.uint32)
        st = np.ascontiguousarray(steps, dtype=np.uint64)
        assert len(ids) == len(st)
        check(self.ctx.handle, load().sg_hosts_skip(self.handle, len(ids), ids.ctypes.data, st.ctypes.data))

    def __del__(self):
        try:
            if getattr(self, "handle", None):
                load().sg_hosts_destroy(self.handle)
                self.handle = None
        except Exception:
            pass


class DeviceTable(_Versioned):
    """A routing-table shard resident on the device (rows [row_begin, row_begin + n_rows))."""

    def __init__(self, latency_ns, packet_loss, n_cols: int, row_begin: int = 0):
        torch = _torch()
        assert latency_ns.dtype == torch.int64 and packet_loss.dtype == torch.float32
        self.latency_ns, self.packet_loss = latency_ns, packet_loss
        self.n_cols = int(n_cols)
        self.row_begin = int(row_begin)
        self.n_rows = latency_ns.numel() // max(self.n_cols, 1)
        self.path_key = None  # packed (lat << 32 | bits(loss)) cells, set by pack()

    def pack(self, ctx=None) -> bool:
        """Build the packed path-key copy of the table (sg_table_pack), so a
        delivery round gathers one 8-byte word per packet.  Returns False and
        keeps the two-array form when some latency is 2^32 ns or more."""
        torch = _torch()
        ctx = ctx or default_context()
        key = torch.empty(max(self.latency_ns.numel(), 1), dtype=torch.int64, device=self.latency_ns.device)
        ok = C.c_uint32(0)
        self.path_key = None
        t = self.struct()
        _capi.check(ctx.handle, load().sg_table_pack(ctx.handle, C.byref(t), key.data_ptr(), C.byref(ok)))
        if ok.value:
            self.path_key = key
        return bool(ok.value)

    _FIELDS = ("latency_ns", "packet_loss", "path_key")

    def c_struct(self) -> _capi.sg_table:
        return _cached(self, self._FIELDS, self.struct)



    def struct(self) -> _capi.sg_table:
        t = _capi.sg_table()
        t.latency_ns = self.latency_ns.data_ptr()
        t.packet_loss = self.packet_loss.data_ptr()
        t.n_cols, t.row_begin, t.n_rows = self.n_cols, self.row_begin, self.n_rows
        t.path_key = self.path_key.data_ptr() if self.path_key is not None else None
        return t


@dataclass
class PacketBatch(_Versioned):
    """One round's sends, grouped by ascending source host, each host's packets in send order."""

    src_host: "object"     # int32 device tensor (u32 bits)
    dst_ipv4: "object"     # int32 device tensor (u32 bits)
    payload_len: "object"  # int32 device tensor
    send_time_ns: "object"  # int64 device tensor (u64 bits)
    # int32 device tensor (u32 bits) or None: RNG steps the source host's other
    # consumers (syscalls, host.rs:645-647) took since its previous packet (sg_packets.rng_skip)
    rng_skip: "object" = None

    @classmethod
    def from_numpy(cls, src_host, dst_ipv4, payload_len, send_time_ns, device="cuda", rng_skip=None):
        return cls(_dev_u32(src_host, device), _dev_u32(dst_ipv4, device), _dev_u32(payload_len, device),
                   _dev_u64(send_time_ns, device), None if rng_skip is None else _dev_u32(rng_skip, device))

    def __len__(self):
        return int(self.src_host.numel())

    def c_struct(self) -> _capi.sg_packets:
        def build():
            p = _capi.sg_packets()
            p.n_packets = len(self)
            p.src_host, p.dst_ipv4 = self.src_host.data_ptr(), self.dst_ipv4.data_ptr()
            p.payload_len, p.send_time_ns = self.payload_len.data_ptr(), self.send_time_ns.data_ptr()
            if self.rng_skip is not None:
                _capi.require_abi(5, "PacketBatch.rng_skip")
            p.rng_skip = self.rng_skip.data_ptr() if self.rng_skip is not None else None
            return p

        return _cached(self, self._FIELDS, build)

    _FIELDS = ("src_host", "dst_ipv4", "payload_len", "send_time_ns", "rng_skip")




@dataclass
class Deliveries(_Versioned):
    status: "object"          # uint8 device tensor (SG_PKT_*)
    deliver_time_ns: "object"  # int64 (u64 bits)
    event_id: "object"        # int64 (u64 bits; -1 = none)
    dst_order: "object"       # int32
    dst_offsets: "object"     # int32, n_hosts + 1
    n_delivered: int = 0
    min_deliver_time_ns: int = 0
    min_used_latency_ns: int = 0

    @classmethod
    def allocate(cls, n_packets: int, n_hosts: int, device="cuda"):
        torch = _torch()
        return cls(torch.empty(max(n_packets, 1), dtype=torch.uint8, device=device),
                   torch.empty(max(n_packets, 1), dtype=torch.int64, device=device),
                   torch.empty(max(n_packets, 1), dtype=torch.int64, device=device),
                   torch.empty(max(n_packets, 1), dtype=torch.int32, device=device),
                   torch.empty(n_hosts + 1, dtype=torch.int32, device=device))

    def c_struct(self) -> _capi.sg_deliveries:
        def build():
            d = _capi.sg_deliveries()
            d.status, d.deliver_time_ns = self.status.data_ptr(), self.deliver_time_ns.data_ptr()
            d.event_id, d.dst_order = self.event_id.data_ptr(), self.dst_order.data_ptr()
            d.dst_offsets = self.dst_offsets.data_ptr()
            return d

        return _cached(self, self._FIELDS, build)

    _FIELDS = ("status", "deliver_time_ns", "event_id", "dst_order", "dst_offsets")



    def to_numpy(self, n_packets: int) -> dict:
        nd = self.n_delivered
        return dict(status=self.status[:n_packets].cpu().numpy(),
                    deliver_time=self.deliver_time_ns[:n_packets].cpu().numpy().view(np.uint64),
                    event_id=self.event_id[:n_packets].cpu().numpy().view(np.uint64),
                    dst_order=self.dst_order[:nd].cpu().numpy().view(np.uint32),
                    dst_offsets=self.dst_offsets.cpu().numpy().view(np.uint32),
                    min_deliver=self.min_deliver_time_ns, min_lat=self.min_used_latency_ns,
                    delivered=nd)


def deliver_round(hosts: HostTable, table: DeviceTable, packets: PacketBatch, round_end_ns: int,
                  sim_end_ns: int, bootstrap_end_ns: int = 0, out: Optional[Deliveries] = None,
                  ctx: Optional[Context] = None) -> Deliveries:
    """One round of Worker::send_packet + push_packet_to_host for every logged packet.

    A round loop that passes the same objects again reuses the call's ctypes arguments (the
    structs are rebuilt only when one of their tensors is replaced): the wrapper then costs a few
    microseconds per round, which the Rust caller of INTEGRATION.md does not pay at all."""
    ctx = ctx or hosts.ctx
    if out is not None:
        plan = out.__dict__.get("_plan")
        if plan is not None and plan[0]() is hosts and plan[1]() is table and plan[2]() is packets and plan[3] is ctx \
                and plan[4] == table.c_struct_key() and plan[5] == packets.c_struct_key() \
                and plan[6] == out.c_struct_key():
            r, st, args = plan[7], plan[8], plan[9]
            r.round_end_ns, r.sim_end_ns, r.bootstrap_end_ns = round_end_ns, sim_end_ns, bootstrap_end_ns
            check(args[0], _DELIVER_ROUND[0](*args))
            out.n_delivered = st.n_delivered
            out.min_deliver_time_ns = st.min_deliver_time_ns
            out.min_used_latency_ns = st.min_used_latency_ns
            return out
    n = len(packets)
    out = out or Deliveries.allocate(n, hosts.n, device=packets.src_host.device if n else "cuda")
    if out.status.numel() < n or out.dst_offsets.numel() < hosts.n + 1:
        raise ValueError("Deliveries buffers are smaller than the round")
    p = packets.c_struct()
    d = out.c_struct()
    t = table.c_struct()
    r = _capi.sg_round(round_end_ns, sim_end_ns, bootstrap_end_ns)
    st = _capi.sg_round_stats()
    if _DELIVER_ROUND[0] is None:
        _DELIVER_ROUND[0] = load().sg_deliver_round
    args = (ctx.handle, hosts.handle, C.byref(t), C.byref(r), C.byref(p), C.byref(d), C.byref(st))
    check(ctx.handle, _DELIVER_ROUND[0](*args))
    # (weak references: a cached plan must not keep a round's table or batch alive)
    out.__dict__["_plan"] = (weakref.ref(hosts), weakref.ref(table), weakref.ref(packets), ctx,
                             table.c_struct_key(), packets.c_struct_key(),
                             out.c_struct_key(), r, st, args, t, p, d)
    out.n_delivered = st.n_delivered
    out.min_deliver_time_ns = st.min_deliver_time_ns
    out.min_used_latency_ns = st.min_used_latency_ns
    return out


_DELIVER_ROUND = [None]  # the bound entry point (looked up once)
