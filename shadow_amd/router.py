"""Routers' inbound CoDel queues on the device: host-side mirror of
Router::inbound_packets (src/main/network/router/mod.rs:15-58) and
CoDelQueue (src/main/network/router/codel_queue.rs); and the inbound pipeline
(`InboundPipeline`): router queue -> relay_inet_in token bucket
(src/main/network/relay/mod.rs, relay/token_bucket.rs); and the outbound
pipeline (`OutboundPipeline`): interface fifo -> relay_inet_out token bucket ->
router -> Worker::send_packet, whose output is a delivery round's PacketBatch.

One queue per host lives on the device across calls.  `CoDelQueues.run`
applies a batch of push / pop events -- grouped by ascending host, each host's
in the order the host performed them -- exactly as the reference's
`CoDelQueue::push(packet, now)` / `CoDelQueue::pop(now)` would, one device
lane per host.  Every computation is the HIP kernel in libshadow_gpu.so.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import _capi
from ._capi import check, load
from .graph import Context, default_context

PUSH, POP = 0, 1                       # SG_CODEL_PUSH / SG_CODEL_POP
QUEUED, DEQUEUED, DROPPED = 0, 1, 2    # SG_CODEL_* packet status
NONE = 0xFFFFFFFF
TARGET_NS = 10_000_000                 # codel_queue.rs:23
INTERVAL_NS = 100_000_000              # codel_queue.rs:28


def _torch():
    import torch

    return torch


def _dev(x, np_dtype, torch_view, device):
    torch = _torch()
    if isinstance(x, torch.Tensor):
        assert x.is_cuda and x.is_contiguous()
        return x
    a = np.ascontiguousarray(np.asarray(x, dtype=np_dtype))
    return torch.from_numpy(a.view(torch_view)).to(device)


@dataclass
class CoDelEvents:
    """One batch of queue operations (device SoA)."""

    host: "object"     # int32 (u32 bits), grouped by ascending host
    kind: "object"     # uint8: PUSH / POP
    time_ns: "object"  # int64 (u64 bits): EmulatedTime of the operation
    packet: "object"   # int32 (u32 bits): the caller's packet id (pushes)
    length: "object"   # int32: PacketRc::len() (pushes)

    @classmethod
    def from_numpy(cls, host, kind, time_ns, packet, length, device="cuda"):
        return cls(_dev(host, np.uint32, np.int32, device), _dev(kind, np.uint8, np.uint8, device),
                   _dev(time_ns, np.uint64, np.int64, device), _dev(packet, np.uint32, np.int32, device),
                   _dev(length, np.uint32, np.int32, device))

    def __len__(self):
        return int(self.host.numel())


class CoDelQueues:
    """The inbound CoDel queue of every host (sg_codel_*)."""

    def __init__(self, n_hosts: int, ring_cap: int = 4096, ctx: Optional[Context] = None):
        self.ctx = ctx or default_context()
        self.n = int(n_hosts)
        h = C.c_void_p()
        check(self.ctx.handle, load().sg_codel_create(self.ctx.handle, self.n, int(ring_cap), C.byref(h)))
        self.handle = h
        self.cap = int(load().sg_codel_ring_cap(h))

    def run(self, ev: CoDelEvents, pkt_status, n_packets: Optional[int] = None):
        """Apply the events.  pkt_status (uint8 device tensor indexed by packet id) is
        set to DEQUEUED / DROPPED as packets leave.  Returns (pop_result int32 device
        tensor: the popped packet or NONE per event, packets dropped)."""
        torch = _torch()
        n = len(ev)
        res = torch.empty(max(n, 1), dtype=torch.int32, device=ev.host.device)
        e = _capi.sg_codel_events(n, ev.host.data_ptr(), ev.kind.data_ptr(), ev.time_ns.data_ptr(),
                                  ev.packet.data_ptr(), ev.length.data_ptr())
        nd = C.c_uint64()
        ns = int(pkt_status.numel()) if n_packets is None else int(n_packets)
        check(self.ctx.handle, load().sg_codel_run(self.ctx.handle, self.handle, C.byref(e), res.data_ptr(),
                                                   pkt_status.data_ptr(), ns, C.byref(nd)))
        return res[:n], int(nd.value)

    def get_state(self) -> dict:
        """Per-host state (the oracle's layout: flags, interval_end, drop_next, cur, prev,
        bytes, head, tail, ring_pkt, ring_ts, ring_len)."""
        n, r = self.n, self.n * self.cap
        st = dict(cap=self.cap, flags=np.zeros(n, np.uint8), interval_end=np.zeros(n, np.uint64),
                  drop_next=np.zeros(n, np.uint64), cur=np.zeros(n, np.uint64), prev=np.zeros(n, np.uint64),
                  bytes=np.zeros(n, np.uint64), head=np.zeros(n, np.uint32), tail=np.zeros(n, np.uint32),
                  ring_pkt=np.zeros(r, np.uint32), ring_ts=np.zeros(r, np.uint64), ring_len=np.zeros(r, np.uint32))
        check(self.ctx.handle, load().sg_codel_get_state(self.handle, C.byref(self._struct(st))))
        return st

    def set_state(self, st: dict) -> None:
        check(self.ctx.handle, load().sg_codel_set_state(self.handle, C.byref(self._struct(st))))

    @staticmethod
    def _struct(st) -> _capi.sg_codel_state:
        v = lambda a: a.ctypes.data_as(C.c_void_p)
        return _capi.sg_codel_state(v(st["flags"]), v(st["interval_end"]), v(st["drop_next"]), v(st["cur"]),
                                    v(st["prev"]), v(st["bytes"]), v(st["head"]), v(st["tail"]),
                                    v(st["ring_pkt"]), v(st["ring_ts"]), v(st["ring_len"]))

    def __del__(self):
        try:
            if getattr(self, "handle", None):
                load().sg_codel_destroy(self.handle)
                self.handle = None
        except Exception:
            pass


class InboundPipeline:
    """Every host's router CoDel queue + inbound relay (sg_inbound_*): arrivals (a
    delivery round's buckets) are pushed and forwarded to the interface as each
    host's token bucket allows; forward tasks past a window's end stay pending."""

    def __init__(self, bw_down_bits, ring_cap: int = 4096, ctx: Optional[Context] = None):
        self.ctx = ctx or default_context()
        bw = np.ascontiguousarray(bw_down_bits, dtype=np.uint64)
        self.n = len(bw)
        h = C.c_void_p()
        check(self.ctx.handle, load().sg_inbound_create(self.ctx.handle, self.n, bw.ctypes.data, int(ring_cap),
                                                        C.byref(h)))
        self.handle = h
        self.cap = int(load().sg_inbound_ring_cap(h))

    def run(self, host, time_ns, packet, length, window_end_ns: int, bootstrap_end_ns: int, sim_end_ns: int,
            fwd_time, pkt_status, event_ctr_ptr: Optional[int] = None) -> int:
        """Arrivals as device tensors (int32 host/packet/length, int64 time); fwd_time (int64)
        and pkt_status (uint8) are indexed by packet id.  Returns the CoDel drops."""
        n = int(host.numel())
        a = _capi.sg_inbound_arrivals(n, host.data_ptr(), time_ns.data_ptr(), packet.data_ptr(), length.data_ptr())
        nd = C.c_uint64()
        check(self.ctx.handle, load().sg_inbound_run(self.ctx.handle, self.handle, C.byref(a), int(window_end_ns),
                                                     int(bootstrap_end_ns), int(sim_end_ns),
                                                     C.c_void_p(event_ctr_ptr or 0), fwd_time.data_ptr(),
                                                     pkt_status.data_ptr(), int(pkt_status.numel()), C.byref(nd)))
        return int(nd.value)

    def run_ordered(self, host, time_ns, packet, length, window_end_ns: int, bootstrap_end_ns: int,
                    sim_end_ns: int, fwd_time, pkt_status, arr_fwd_time, arr_status,
                    event_ctr_ptr: Optional[int] = None) -> int:
        """run() with this call's arrivals' fates in arrival order (sg_inbound_run_ordered):
        arr_status (uint8, zeroed by the caller) and arr_fwd_time (int64), one per arrival;
        packets from earlier calls that leave now still go to fwd_time / pkt_status by id."""
        n = int(host.numel())
        if n and (arr_status.numel() < n or arr_fwd_time.numel() < n):
            raise ValueError("arrival outputs shorter than the arrivals")
        a = _capi.sg_inbound_arrivals(n, host.data_ptr(), time_ns.data_ptr(), packet.data_ptr(), length.data_ptr())
        nd = C.c_uint64()
        check(self.ctx.handle, load().sg_inbound_run_ordered(
            self.ctx.handle, self.handle, C.byref(a), int(window_end_ns), int(bootstrap_end_ns), int(sim_end_ns),
            C.c_void_p(event_ctr_ptr or 0), fwd_time.data_ptr() if fwd_time is not None else None,
            pkt_status.data_ptr() if pkt_status is not None else None,
            int(pkt_status.numel()) if pkt_status is not None else 0, arr_fwd_time.data_ptr(), arr_status.data_ptr(),
            C.byref(nd)))
        return int(nd.value)

    def get_state(self) -> dict:
        """Queue state (CoDelQueues.get_state layout) + relay state (the oracle's inbound_state keys)."""
        n = self.n
        st = dict(cap=self.cap, flags=np.zeros(n, np.uint8), interval_end=np.zeros(n, np.uint64),
                  drop_next=np.zeros(n, np.uint64), cur=np.zeros(n, np.uint64), prev=np.zeros(n, np.uint64),
                  bytes=np.zeros(n, np.uint64), head=np.zeros(n, np.uint32), tail=np.zeros(n, np.uint32),
                  ring_pkt=np.zeros(n * self.cap, np.uint32), ring_ts=np.zeros(n * self.cap, np.uint64),
                  ring_len=np.zeros(n * self.cap, np.uint32), rflags=np.zeros(n, np.uint8),
                  task_time=np.zeros(n, np.uint64), task_id=np.zeros(n, np.uint64), task_born=np.zeros(n, np.uint64),
                  cached_pkt=np.zeros(n, np.uint32),
                  cached_len=np.zeros(n, np.uint32), tb_cap=np.zeros(n, np.uint64), tb_bal=np.zeros(n, np.uint64),
                  tb_inc=np.zeros(n, np.uint64), tb_last=np.zeros(n, np.uint64))
        v = lambda k: st[k].ctypes.data_as(C.c_void_p)
        rs = _capi.sg_inbound_relay_state(v("rflags"), v("task_time"), v("cached_pkt"), v("cached_len"), v("tb_cap"),
                                          v("tb_bal"), v("tb_inc"), v("tb_last"), v("task_id"), v("task_born"))
        check(self.ctx.handle, load().sg_inbound_get_state(self.handle, C.byref(CoDelQueues._struct(st)),
                                                           C.byref(rs)))
        return st

    def __del__(self):
        try:
            if getattr(self, "handle", None):
                load().sg_inbound_destroy(self.handle)
                self.handle = None
        except Exception:
            pass


class OutboundPipeline:
    """Every host's network interface (fifo qdisc) + outbound relay (sg_outbound_*):
    sends enter the interface in creation order; the relay forwards them as the
    host's token bucket (bw up) allows, packets to the host's own address back to
    the interface, the rest to the router, i.e. to Worker::send_packet.  The
    packets sent form the next delivery round's PacketBatch (`run` returns it)."""

    def __init__(self, host_ipv4, bw_up_bits, ring_cap: int = 4096, ctx: Optional[Context] = None):
        self.ctx = ctx or default_context()
        ip = np.ascontiguousarray(host_ipv4, dtype=np.uint32)
        bw = np.ascontiguousarray(bw_up_bits, dtype=np.uint64)
        assert len(ip) == len(bw)
        self.n = len(bw)
        h = C.c_void_p()
        check(self.ctx.handle, load().sg_outbound_create(self.ctx.handle, self.n, ip.ctypes.data, bw.ctypes.data,
                                                         int(ring_cap), C.byref(h)))
        self.handle = h
        self.cap = int(load().sg_outbound_ring_cap(h))
        self._sent = None

    def sent_buffers(self, cap: int, device):
        """Device buffers for the sent batch (grown, then reused across windows)."""
        import torch
        if self._sent is None or self._sent["src_host"].numel() < cap:
            i32 = dict(dtype=torch.int32, device=device)
            self._sent = dict(src_host=torch.empty(cap, **i32), dst_ipv4=torch.empty(cap, **i32),
                              payload_len=torch.empty(cap, **i32),
                              send_time_ns=torch.empty(cap, dtype=torch.int64, device=device),
                              packet=torch.empty(cap, **i32))
        return self._sent

    def run(self, host, time_ns, packet, length, payload_len, dst_ipv4, window_end_ns: int, bootstrap_end_ns: int,
            sim_end_ns: int, fwd_time, pkt_status, event_ctr_ptr: Optional[int] = None, sent_cap: Optional[int] = None,
            event_id=None, event_created_ns=None, collect: bool = True):
        """Sends as device tensors (int32 host/packet/length/payload_len/dst_ipv4, int64 time); fwd_time
        (int64) and pkt_status (uint8) are indexed by packet id.  event_id / event_created_ns (int64
        device tensors, optional, together; they need event_ctr_ptr): the sending event's id (-1 =
        UINT64_MAX: a Packet event) and creation time, which order a send against a forward task at
        the same time (sg_outbound_sends).  Returns (PacketBatch of the packets sent, in send_packet
        order, and their packet ids), views of buffers reused by the next call; with collect=False no
        sent batch is written (sent = NULL) and it returns (None, the number of packets sent)."""
        from .worker import PacketBatch
        n = int(host.numel())
        keyed = event_id is not None
        if keyed:
            _capi.require_abi(6, "OutboundPipeline.run with event ids")
        s = _capi.sg_outbound_sends(n, host.data_ptr(), time_ns.data_ptr(), packet.data_ptr(), length.data_ptr(),
                                    payload_len.data_ptr(), dst_ipv4.data_ptr(),
                                    event_id.data_ptr() if keyed else None,
                                    event_created_ns.data_ptr() if event_created_ns is not None else None)
        ns = C.c_uint32()
        if not collect:
            check(self.ctx.handle, load().sg_outbound_run(self.ctx.handle, self.handle, C.byref(s),
                                                          int(window_end_ns), int(bootstrap_end_ns), int(sim_end_ns),
                                                          C.c_void_p(event_ctr_ptr or 0), fwd_time.data_ptr(),
                                                          pkt_status.data_ptr(), int(pkt_status.numel()), None,
                                                          C.byref(ns)))
            return None, ns.value
        cap = int(sent_cap if sent_cap is not None else n + self.n * 4)
        b = self.sent_buffers(max(cap, 1), fwd_time.device)
        o = _capi.sg_outbound_sent(cap, *(b[k].data_ptr() for k in ("src_host", "dst_ipv4", "payload_len",
                                                                     "send_time_ns", "packet")))
        check(self.ctx.handle, load().sg_outbound_run(self.ctx.handle, self.handle, C.byref(s), int(window_end_ns),
                                                      int(bootstrap_end_ns), int(sim_end_ns),
                                                      C.c_void_p(event_ctr_ptr or 0), fwd_time.data_ptr(),
                                                      pkt_status.data_ptr(), int(pkt_status.numel()), C.byref(o),
                                                      C.byref(ns)))
        k = ns.value
        batch = PacketBatch(b["src_host"][:k], b["dst_ipv4"][:k], b["payload_len"][:k], b["send_time_ns"][:k])
        return batch, b["packet"][:k]

    def get_state(self) -> dict:
        """Queue + relay state in the oracle's outbound_state layout (cached packet = slot head - 1)."""
        n, c = self.n, self.cap
        st = dict(cap=c, head=np.zeros(n, np.uint32), tail=np.zeros(n, np.uint32),
                  ring_pkt=np.zeros(n * c, np.uint32), ring_len=np.zeros(n * c, np.uint32),
                  ring_pay=np.zeros(n * c, np.uint32), ring_dst=np.zeros(n * c, np.uint32),
                  rflags=np.zeros(n, np.uint8), task_time=np.zeros(n, np.uint64), task_id=np.zeros(n, np.uint64),
                  task_born=np.zeros(n, np.uint64), tb_cap=np.zeros(n, np.uint64),
                  tb_bal=np.zeros(n, np.uint64), tb_inc=np.zeros(n, np.uint64), tb_last=np.zeros(n, np.uint64))
        v = lambda k: st[k].ctypes.data_as(C.c_void_p)
        q = _capi.sg_outbound_queue_state(v("head"), v("tail"), v("ring_pkt"), v("ring_len"), v("ring_pay"),
                                          v("ring_dst"))
        rs = _capi.sg_inbound_relay_state(v("rflags"), v("task_time"), None, None, v("tb_cap"), v("tb_bal"),
                                          v("tb_inc"), v("tb_last"), v("task_id"), v("task_born"))
        check(self.ctx.handle, load().sg_outbound_get_state(self.handle, C.byref(q), C.byref(rs)))
        return st

    def __del__(self):
        try:
            if getattr(self, "handle", None):
                load().sg_outbound_destroy(self.handle)
                self.handle = None
        except Exception:
            pass
