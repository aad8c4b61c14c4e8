"""Multi-GPU sharding of the network core: one process per GPU, RCCL over xGMI.

Routing build: source rows are independent problems.  Rank r computes rows
`row_range(n_used, world, r)`; the graph (a few MB) is replicated.  When a
replicated table is wanted, the row blocks are all-gathered (equal block sizes,
padded), otherwise each rank keeps its shard -- which is all delivery needs,
because a packet only reads its source host's row.

Delivery: hosts are owned by the rank that holds their routing row
(`HostPartition`).  Each round:
  1. source phase on every rank (sg_deliver_source): the send_packet half for
     the packets its hosts sent, records packed by destination owner;
  2. all-to-all of the per-rank record counts, then of the records
     (32 B each).  With a comm.Comm in place of `dist` (the default on RCCL
     process groups) every exchange is a call into the library (sg_comm_*,
     RCCL on the context's stream), the same calls the Rust caller makes
     (INTEGRATION.md); torch.distributed remains for gloo rehearsals;
  3. destination phase (sg_deliver_bucket): per-destination EventQueue order.
With `padded=True` (ShardedDelivery) the rounds after the first use a
fixed-split exchange with no host round trip before the round's end: every
rank's records for rank r fill a block of `cap` slots (sg_deliver_source_padded),
one all-gather of each rank's [stats, counts] row and one equal-split
all-to-all move them, and the bucketing reads the valid records of each block
(sg_deliver_bucket_padded), which synchronises once.  cap follows the largest
pair count of the round before (all ranks see the same gathered rows, so they
agree on it); a round whose counts outgrow it is exchanged again exactly.
The phases are injectable so the exchange logic is testable on CPU (gloo).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence

import numpy as np

from . import _capi
from ._capi import check, load
from .comm import is_comm

NONE = 0xFFFFFFFF
RECORD_DTYPE = np.dtype([("deliver_time_ns", "<u8"), ("order_key", "<u8"), ("event_id", "<u8"),
                         ("packet", "<u4"), ("dst_host", "<u4")])
assert RECORD_DTYPE.itemsize == 32


def row_range(n_used: int, world: int, rank: int):
    """Contiguous, equal-size (last one short) row block of `rank`."""
    per = (n_used + world - 1) // max(world, 1)
    return min(rank * per, n_used), min((rank + 1) * per, n_used), per


def balanced_node_order(host_node: Sequence[int], n_nodes: int, world: int, host_weight=None, tol=0.05):
    """Row order of the used nodes that balances delivery across `world` rank blocks.

    A host is owned by the rank holding its node's routing row, so with the identity
    order a skewed host map (many hosts on a few nodes, as on a Tor-like graph) puts
    most senders on one rank.  Here nodes are dealt to ranks largest weight first
    (weight = the summed host_weight of their hosts, 1 per host by default), each
    to the lightest rank that still has room for a full row block, and then ordered
    by rank: every rank still builds an equal block of rows, now with an even share
    of the senders.  A single node heavier than a rank's share cannot be split (its
    hosts share one routing row) and bounds the balance.

    When the identity order is already balanced (every rank's share within `tol` of
    the mean) it is kept: a rank's row block is then a run of consecutive node ids,
    which in a graph numbered with any locality (a ring, a geographic order) holds
    neighbours of its own rows -- the bound rows a block's search plans from
    (sg_routing.hip, flagged plan).  Dealt by weight, equal weights go round-robin and
    a block holds almost no neighbours of its rows, so most of its rows search from
    infinity (C3 at N = 2: 2.36 against 1.93 ms per block, tools/sssp_ab.py --rows).

    Returns (order, route): order[i] = node index of table row i (the `used` list to
    build with), route[h] = table row of host h's node."""
    host_node = np.asarray(host_node, dtype=np.int64)
    w = np.bincount(host_node, weights=None if host_weight is None else np.asarray(host_weight, np.float64),
                    minlength=n_nodes).astype(np.float64)
    per = (n_nodes + world - 1) // max(world, 1)
    ident = np.array([w[r * per:(r + 1) * per].sum() for r in range(world)])
    if world <= 1 or ident.max() <= (1.0 + tol) * max(ident.mean(), 1e-300):
        order = np.arange(n_nodes, dtype=np.uint32)
        return order, host_node.astype(np.uint32)
    cap = [min(per, max(0, n_nodes - r * per)) for r in range(world)]
    load = np.zeros(world)
    fill = np.zeros(world, np.int64)
    rank_of = np.empty(n_nodes, np.int64)
    for v in np.argsort(-w, kind="stable"):  # heaviest first, ties by node index
        open_ = np.nonzero(fill < cap)[0]
        r = open_[np.argmin(load[open_])]
        rank_of[v] = r
        load[r] += w[v]
        fill[r] += 1
    order = np.argsort(rank_of, kind="stable").astype(np.uint32)
    pos = np.empty(n_nodes, np.uint32)
    pos[order] = np.arange(n_nodes, dtype=np.uint32)
    return order, pos[host_node]


class HostPartition:
    """owner[h] = rank holding host h's routing row; local[h] = slot on its owner.
    Rows are split in equal blocks (row_range); balanced_node_order chooses a row
    order whose blocks carry even shares of the hosts."""

    def __init__(self, host_route: Sequence[int], n_used: int, world: int):
        route = np.asarray(host_route, dtype=np.int64)
        per = (n_used + world - 1) // max(world, 1)
        self.world = world
        self.owner = (route // per).astype(np.uint32)
        self.hosts_of = [np.nonzero(self.owner == r)[0].astype(np.uint32) for r in range(world)]
        self.local = np.full(len(route), NONE, np.uint32)
        for r in range(world):
            self.local[self.hosts_of[r]] = np.arange(len(self.hosts_of[r]), dtype=np.uint32)

    def n_local(self, rank: int) -> int:
        return len(self.hosts_of[rank])


class Workspace:
    """Round buffers kept across rounds: `get` returns the first `n` elements of a
    cached tensor, reallocated only when a round needs more.  Reuse across rounds
    is stream-ordered: every kernel runs on the current stream, and the blocking
    collectives (async_op=False) make that stream wait for RCCL's."""

    def __init__(self):
        self._t = {}

    def get(self, name, n, dtype, device, cols=None, pinned=False):
        import torch

        shape = (n,) if cols is None else (n, cols)
        t = self._t.get(name)
        if t is None or t.shape[0] < n or t.dtype != dtype or str(t.device) != str(device):
            cap = max(n, 1) if t is None else max(n, 1, t.shape[0] + t.shape[0] // 2)
            full = (cap,) if cols is None else (cap, cols)
            t = torch.empty(full, dtype=dtype, device=device, pin_memory=pinned)
            self._t[name] = t
        return t[:n] if shape[0] else t[:0]


# ---------------------------------------------------------------------------
# GPU phases (libshadow_gpu.so)
# ---------------------------------------------------------------------------
@dataclass
class SourceResult:
    """A rank's source phase of one round.  In a padded round (ShardedDelivery(padded=True),
    every round after the first) the records are the blocks `send_padded` ([n_ranks * cap, 4],
    rank r's block at r * cap, min(count, cap) valid records each) and `send` is None: the compact
    array is complete only when the round overflowed into an exact exchange (last_mode
    "padded+exact"), where `send` holds it.  Read records of a padded round from send_padded, or
    call gpu_pad_to_compact for the compact form."""
    status: object           # uint8 device tensor
    deliver_time_ns: object  # int64 device tensor
    event_id: object         # int64 device tensor
    send: object             # int64 device tensor [n, 4] (sg_record)
    send_counts: List[int]
    n_delivered: int
    min_deliver_time_ns: int
    min_used_latency_ns: int
    send_padded: object = None  # padded rounds: the [n_ranks * cap, 4] blocks (send is then None
    #                             unless the round overflowed into an exact exchange)


def gpu_source_phase(ctx, hosts, table, packets, round_end_ns, sim_end_ns, bootstrap_end_ns, owner_dev,
                     n_ranks, ws: Optional[Workspace] = None) -> SourceResult:
    import torch

    n = len(packets)
    dev = packets.src_host.device
    if ws is None:
        ws = Workspace()
    status = ws.get("status", max(n, 1), torch.uint8, dev)
    deliver = ws.get("deliver", max(n, 1), torch.int64, dev)
    eid = ws.get("eid", max(n, 1), torch.int64, dev)
    send = ws.get("send", max(n, 1), torch.int64, dev, cols=4)
    counts = (C.c_uint32 * n_ranks)()
    p = _capi.sg_packets()
    p.n_packets = n
    p.src_host, p.dst_ipv4 = packets.src_host.data_ptr(), packets.dst_ipv4.data_ptr()
    p.payload_len, p.send_time_ns = packets.payload_len.data_ptr(), packets.send_time_ns.data_ptr()
    skip = getattr(packets, "rng_skip", None)
    p.rng_skip = skip.data_ptr() if skip is not None else None
    r = _capi.sg_round(round_end_ns, sim_end_ns, bootstrap_end_ns)
    st = _capi.sg_round_stats()
    t = table.struct()
    check(ctx.handle, load().sg_deliver_source(ctx.handle, hosts.handle, C.byref(t), C.byref(r), C.byref(p),
                                               status.data_ptr(), deliver.data_ptr(), eid.data_ptr(),
                                               owner_dev.data_ptr(), n_ranks, send.data_ptr(), counts,
                                               C.byref(st)))
    return SourceResult(status, deliver, eid, send, list(counts), st.n_delivered, st.min_deliver_time_ns,
                        st.min_used_latency_ns)


def gpu_bucket_phase(ctx, recv, n_records: int, local_dev, n_hosts: int, n_local: int,
                     ws: Optional[Workspace] = None):
    import torch

    dev = local_dev.device
    if ws is None:
        ws = Workspace()
    order = ws.get("order", max(n_records, 1), torch.int32, dev)
    offsets = ws.get("offsets", n_local + 1, torch.int32, dev)
    check(ctx.handle, load().sg_deliver_bucket(ctx.handle, recv.data_ptr() if n_records else None, n_records,
                                               local_dev.data_ptr(), n_hosts, n_local, order.data_ptr(),
                                               offsets.data_ptr()))
    return order[:n_records], offsets


@dataclass
class SourcePadded:
    status: object
    deliver_time_ns: object
    event_id: object
    send_padded: object  # int64 device tensor [n_ranks * cap, 4] (sg_record blocks)
    send: object         # int64 device tensor [n, 4]: records past cap at their compact positions
    xrow: object         # int64 device tensor [3 + n_ranks]: stats, then the count for each rank
    cap: int


def gpu_source_phase_padded(ctx, hosts, table, packets, round_end_ns, sim_end_ns, bootstrap_end_ns, owner_dev,
                            n_ranks, cap, ws: Optional[Workspace] = None) -> SourcePadded:
    import torch

    n = len(packets)
    dev = packets.src_host.device
    ws = ws or Workspace()
    status = ws.get("status", max(n, 1), torch.uint8, dev)
    deliver = ws.get("deliver", max(n, 1), torch.int64, dev)
    eid = ws.get("eid", max(n, 1), torch.int64, dev)
    send = ws.get("send", max(n, 1), torch.int64, dev, cols=4)
    padded = ws.get("send_padded", n_ranks * cap, torch.int64, dev, cols=4)
    xrow = ws.get("xrow", 3 + n_ranks, torch.int64, dev)
    p = _capi.sg_packets()
    p.n_packets = n
    p.src_host, p.dst_ipv4 = packets.src_host.data_ptr(), packets.dst_ipv4.data_ptr()
    p.payload_len, p.send_time_ns = packets.payload_len.data_ptr(), packets.send_time_ns.data_ptr()
    skip = getattr(packets, "rng_skip", None)
    p.rng_skip = skip.data_ptr() if skip is not None else None
    r = _capi.sg_round(round_end_ns, sim_end_ns, bootstrap_end_ns)
    t = table.struct()
    check(ctx.handle, load().sg_deliver_source_padded(ctx.handle, hosts.handle, C.byref(t), C.byref(r), C.byref(p),
                                                      status.data_ptr(), deliver.data_ptr(), eid.data_ptr(),
                                                      owner_dev.data_ptr(), n_ranks, cap, padded.data_ptr(),
                                                      send.data_ptr(), xrow.data_ptr()))
    return SourcePadded(status, deliver, eid, padded, send, xrow, cap)


def gpu_bucket_phase_padded(ctx, recv_padded, cap: int, xall, rank: int, local_dev, n_hosts: int, n_local: int,
                            ws: Optional[Workspace] = None):
    """Returns (order into recv_padded, offsets, global stats, recv_counts, pair_max)."""
    import torch

    dev = local_dev.device
    ws = ws or Workspace()
    n_ranks = recv_padded.shape[0] // cap
    order = ws.get("order", max(n_ranks * cap, 1), torch.int32, dev)
    offsets = ws.get("offsets", n_local + 1, torch.int32, dev)
    st = _capi.sg_round_stats()
    rc = (C.c_uint32 * n_ranks)()
    pm = C.c_uint32()
    check(ctx.handle, load().sg_deliver_bucket_padded(ctx.handle, recv_padded.data_ptr(), n_ranks, cap, xall.data_ptr(),
                                                      rank, local_dev.data_ptr(), n_hosts, n_local, order.data_ptr(),
                                                      offsets.data_ptr(), C.byref(st), rc, C.byref(pm)))
    counts = list(rc)
    stats = (st.n_delivered, st.min_deliver_time_ns, st.min_used_latency_ns)
    return order[:sum(min(c, cap) for c in counts)], offsets, stats, counts, pm.value


def gpu_pad_to_compact(ctx, src: SourcePadded, n_ranks: int):
    check(ctx.handle, load().sg_deliver_pad_to_compact(ctx.handle, src.send_padded.data_ptr(), n_ranks, src.cap,
                                                       src.xrow.data_ptr(), src.send.data_ptr()))
    return src.send


def _stream_wait(waiter: int, producer: int) -> None:
    """Make stream `waiter` wait for the work enqueued on stream `producer` so far (a HIP
    event; streams as hipStream_t ints, 0 = the legacy default stream).  A no-op for one
    stream."""
    if waiter == producer:
        return
    import torch

    ev = torch.cuda.Event()
    ev.record(torch.cuda.ExternalStream(producer))
    torch.cuda.ExternalStream(waiter).wait_event(ev)


def _streams(ctx, tensor):
    """(the library context's stream, torch's current stream) for device tensors, else None."""
    if ctx is None or not hasattr(ctx, "stream") or getattr(tensor, "device", None) is None \
            or tensor.device.type != "cuda":
        return None
    import torch

    return int(ctx.stream), int(torch.cuda.current_stream(tensor.device).cuda_stream)


def next_cap(pair_max: int) -> int:
    """Block size of the next fixed-split exchange: 1.25x the largest pair count seen,
    plus slack, in whole 256-record units (every rank computes it from the same
    gathered rows, so every rank picks the same value)."""
    return max(256, (int(pair_max) * 5 // 4 + 256 + 255) // 256 * 256)


# ---------------------------------------------------------------------------
# Exchange
# ---------------------------------------------------------------------------
def _comm_in(comm, t) -> None:
    """The library's stream waits for torch's current stream (which wrote `t`)."""
    st = _streams(comm.ctx, t)
    if st:
        _stream_wait(st[0], st[1])


def _comm_out(comm, t) -> None:
    """torch's current stream waits for the library's stream (which wrote `t`)."""
    st = _streams(comm.ctx, t)
    if st:
        _stream_wait(st[1], st[0])


def exchange_padded(send_padded, xrow, dist, group=None, ws: Optional[Workspace] = None):
    """The fixed-split exchange: one all-gather of the [stats, counts] rows and one
    equal-split all-to-all of the record blocks, both enqueued on the stream with no
    host round trip.  `dist` is a comm.Comm (sg_comm_exchange_padded in the library,
    RCCL on the context's stream) or torch.distributed (gloo rehearsals: host-staged).
    Returns (recv_padded, xall)."""
    import torch

    world = dist.get_world_size(group) if dist is not None else 1
    if is_comm(dist):
        ws = ws or Workspace()
        xall = ws.get("xall", world * xrow.shape[0], torch.int64, send_padded.device)
        recv = ws.get("recv_padded", send_padded.shape[0], torch.int64, send_padded.device, cols=4)
        dist.exchange_padded(send_padded, recv, send_padded.shape[0] // max(world, 1), xrow, xall)
        return recv, xall
    if dist is not None and _host_staged(dist, group, send_padded.device):
        recv, xall = exchange_padded(send_padded.cpu(), xrow.cpu(), dist, group)
        return recv.to(send_padded.device), xall.to(send_padded.device)
    ws = ws or Workspace()
    dev = send_padded.device
    xall = ws.get("xall", world * xrow.shape[0], torch.int64, dev)
    recv = ws.get("recv_padded", send_padded.shape[0], torch.int64, dev, cols=4)
    if dist is None:
        xall.copy_(xrow)
        recv.copy_(send_padded)
        return recv, xall
    dist.all_gather_into_tensor(xall, xrow, group=group)
    dist.all_to_all_single(recv, send_padded, group=group)
    return recv, xall
def _host_staged(dist, group, dev) -> bool:
    """gloo moves host tensors only: device tensors go through host copies (the
    multi-rank rehearsal on a box with fewer GPUs than ranks; RCCL needs none)."""
    return not is_comm(dist) and dev.type != "cpu" and dist.get_backend(group) == "gloo"


def all_to_all_records(send, send_counts: List[int], dist, group=None):
    """Counts exchange, then one all_to_all_single of the 32-B records."""
    import torch

    world = len(send_counts)
    if _host_staged(dist, group, send.device):
        recv, counts = all_to_all_records(send.cpu(), send_counts, dist, group)
        return recv.to(send.device), counts
    dev = send.device
    sc = torch.tensor(send_counts, dtype=torch.int64, device=dev)
    rc = torch.empty(world, dtype=torch.int64, device=dev)
    dist.all_to_all_single(rc, sc, group=group)
    recv_counts = [int(x) for x in rc.cpu()]
    return _records_all_to_all(send, send_counts, recv_counts, dist, group), recv_counts


def exchange_round(send, send_counts: List[int], stats, rank: int, dist, group=None,
                   ws: Optional[Workspace] = None, want_pair_max: bool = False):
    """The round's one host round trip: an all-gather of every rank's row
    [delivered, min deliver time, min used latency, counts to each rank] (u64),
    so the round scalars ride with the counts exchange, then the records'
    all_to_all_single.  The row goes up and the gathered rows come back through
    pinned host buffers.  Returns (recv, recv_counts, global stats)."""
    import torch

    world = len(send_counts)
    if _host_staged(dist, group, send.device):
        r = exchange_round(send.cpu(), send_counts, stats, rank, dist, group, want_pair_max=want_pair_max)
        return (r[0].to(send.device),) + tuple(r[1:])
    dev = send.device
    if ws is None:
        ws = Workspace()
    w = 3 + world
    pinned = dev.type != "cpu"
    mine_h = ws.get("x_mine_h", w, torch.int64, "cpu", pinned=pinned)
    mine_h.numpy()[:] = np.array([*stats, *send_counts], dtype=np.uint64).view(np.int64)
    mine_d = ws.get("x_mine_d", w, torch.int64, dev)
    mine_d.copy_(mine_h, non_blocking=True)
    out = ws.get("x_out_d", world * w, torch.int64, dev)
    if is_comm(dist):
        _comm_in(dist, mine_d)
        dist.allgather_u64(mine_d, out)
        _comm_out(dist, out)
    else:
        dist.all_gather_into_tensor(out, mine_d, group=group)
    out_h = ws.get("x_out_h", world * w, torch.int64, "cpu", pinned=pinned)
    out_h.copy_(out, non_blocking=True)
    if pinned:
        torch.cuda.current_stream(dev).synchronize()
    allv = out_h.numpy().view(np.uint64).reshape(world, w)
    recv_counts = [int(allv[r, 3 + rank]) for r in range(world)]
    g = (int(allv[:, 0].sum()), int(allv[:, 1].min()), int(allv[:, 2].min()))
    recv = _records_all_to_all(send, send_counts, recv_counts, dist, group, ws)
    if want_pair_max:
        return recv, recv_counts, g, int(allv[:, 3:].max()) if world else 0
    return recv, recv_counts, g


def _records_all_to_all(send, send_counts: List[int], recv_counts: List[int], dist, group,
                        ws: Optional[Workspace] = None):
    import torch

    dev = send.device
    n_recv = sum(recv_counts)
    recv = (ws or Workspace()).get("x_recv", max(n_recv, 1), torch.int64, dev, cols=4)
    n_send = sum(send_counts)
    if is_comm(dist):
        _comm_in(dist, send)
        dist.alltoallv_records(send, send_counts, recv, recv_counts)
        _comm_out(dist, recv)
        return recv[:n_recv]
    dist.all_to_all_single(recv[:n_recv], send[:n_send], output_split_sizes=recv_counts,
                           input_split_sizes=list(send_counts), group=group)
    return recv[:n_recv]


def gather_round_stats(n_delivered: int, min_deliver: int, min_lat: int, dist, group=None, device="cuda"):
    """Global round scalars (manager.rs:482 next-event minimum, worker.rs:372
    lowest used latency, delivered count): one all-gather of every rank's three
    u64 values (exact for u64; the no-delivery sentinel is UINT64_MAX)."""
    import torch

    mine = np.array([n_delivered, min_deliver, min_lat], dtype=np.uint64).view(np.int64)
    t = torch.from_numpy(mine.copy()).to(device)
    world = dist.get_world_size(group) if dist is not None else 1
    out = torch.empty(3 * world, dtype=torch.int64, device=device)
    if is_comm(dist):
        _comm_in(dist, t)
        dist.allgather_u64(t, out)
        _comm_out(dist, out)
    elif dist is None or world == 1:
        out.copy_(t)
    elif _host_staged(dist, group, out.device):
        host = out.cpu()
        dist.all_gather_into_tensor(host, t.cpu(), group=group)
        out.copy_(host)
    else:
        dist.all_gather_into_tensor(out, t, group=group)
    allv = out.cpu().numpy().view(np.uint64).reshape(world, 3)
    return int(allv[:, 0].sum()), int(allv[:, 1].min()), int(allv[:, 2].min())


def _global_max(v: int, dist, group=None, device="cuda") -> int:
    """max over ranks of one non-negative int (an all-gather of one value per rank)."""
    import torch

    world = dist.get_world_size(group) if dist is not None else 1
    if dist is None or world == 1:
        return int(v)
    if is_comm(dist):
        mine = torch.tensor([int(v)], dtype=torch.int64, device=device)
        out = torch.empty(world, dtype=torch.int64, device=device)
        _comm_in(dist, mine)
        dist.allgather_u64(mine, out)
        _comm_out(dist, out)
        return int(out.max().item())
    dev = "cpu" if _host_staged(dist, group, torch.device(device)) else device
    out = torch.empty(world, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(out, torch.tensor([int(v)], dtype=torch.int64, device=dev), group=group)
    return int(out.max().item())


class ShardedDelivery:
    """One rank's side of a sharded delivery round (see module docstring).

    After round(), last_stats = (delivered, min deliver time, min used latency)
    over all ranks (gather_round_stats)."""

    def __init__(self, ctx, hosts, table, partition: HostPartition, rank: int, world: int, dist=None, group=None,
                 source_fn: Optional[Callable] = None, bucket_fn: Optional[Callable] = None,
                 exchange_fn: Optional[Callable] = None, device="cuda", padded: bool = False,
                 source_padded_fn: Optional[Callable] = None, bucket_padded_fn: Optional[Callable] = None,
                 pad_to_compact_fn: Optional[Callable] = None):
        self.ctx, self.hosts, self.table, self.part = ctx, hosts, table, partition
        self.rank, self.world, self.dist, self.group = rank, world, dist, group
        import functools

        self.ws = Workspace()  # the round's buffers, reused round after round
        self.source_fn = source_fn or functools.partial(gpu_source_phase, ws=self.ws)
        self.bucket_fn = bucket_fn or functools.partial(gpu_bucket_phase, ws=self.ws)
        self.exchange_fn = exchange_fn  # None: exchange_round (counts and round scalars in one all-gather)
        # the fixed-split exchange (rounds after the first: see the module docstring)
        self.padded = padded
        self.source_padded_fn = source_padded_fn or functools.partial(gpu_source_phase_padded, ws=self.ws)
        self.bucket_padded_fn = bucket_padded_fn or functools.partial(gpu_bucket_phase_padded, ws=self.ws)
        self.pad_to_compact_fn = pad_to_compact_fn or gpu_pad_to_compact
        self.cap = None          # block size of the next padded round (None: the next round is exact)
        self.last_mode = None    # "exact", "padded" or "padded+exact" (a padded round that overflowed)
        import torch

        self.owner_dev = torch.from_numpy(partition.owner.view(np.int32)).to(device)
        self.local_dev = torch.from_numpy(partition.local.view(np.int32)).to(device)
        self.device = device
        self.last_stats = None
        self.last = None
        self.last_send_counts = None

    def round(self, packets, round_end_ns: int, sim_end_ns: int, bootstrap_end_ns: int = 0):
        """One round.  The returned tensors are views of buffers the next round
        overwrites (copy what must outlive it).  In a padded round `recv` holds
        n_ranks blocks of `cap` records and `order` indexes it, and the returned
        SourceResult's `send` is None (its records are `send_padded`; see SourceResult)."""
        if self.padded and self.cap is not None:
            return self._round_padded(packets, round_end_ns, sim_end_ns, bootstrap_end_ns)
        out = self._round_exact(packets, round_end_ns, sim_end_ns, bootstrap_end_ns)
        if self.padded:  # the first round sizes the blocks: every rank sees the same counts
            self.cap = next_cap(self._pair_max)
        return out

    def _round_padded(self, packets, round_end_ns, sim_end_ns, bootstrap_end_ns):
        import torch

        cap = self.cap
        src = self.source_padded_fn(self.ctx, self.hosts, self.table, packets, round_end_ns, sim_end_ns,
                                    bootstrap_end_ns, self.owner_dev, self.world, cap)
        # The source phase only enqueues on the library's stream, and the collectives order
        # against torch's current stream: join the two both ways around the exchange (nothing
        # is synchronised until the bucketing's end).
        streams = _streams(self.ctx, src.send_padded)
        if streams:
            _stream_wait(streams[1], streams[0])
        recv, xall = exchange_padded(src.send_padded, src.xrow, self.dist, self.group, ws=self.ws)
        if streams:
            _stream_wait(streams[0], streams[1])
        order, offsets, g, recv_counts, pair_max = self.bucket_padded_fn(
            self.ctx, recv, cap, xall, self.rank, self.local_dev, len(self.part.local), self.part.n_local(self.rank))
        xa = xall.cpu().numpy().view(np.uint64).reshape(self.world, 3 + self.world)  # (after the round's sync)
        send_counts = [int(x) for x in xa[self.rank, 3:]]
        self.last_send_counts = send_counts
        self.last_stats = (int(g[0]), int(g[1]), int(g[2]))
        self.cap = next_cap(pair_max)
        if pair_max > cap:  # some pair outgrew its block: every rank exchanges again, exactly
            self.last_mode = "padded+exact"
            send = self.pad_to_compact_fn(self.ctx, src, self.world)
            recv_counts = [int(xa[b, 3 + self.rank]) for b in range(self.world)]
            recv = _records_all_to_all(send, send_counts, recv_counts, self.dist, self.group, self.ws)
            order, offsets = self.bucket_fn(self.ctx, recv, int(sum(recv_counts)), self.local_dev,
                                            len(self.part.local), self.part.n_local(self.rank))
        else:
            self.last_mode = "padded"
        # a padded round's records are the blocks (records past cap also sit in src.send, at
        # their compact positions; its other slots hold an earlier round's records)
        res = SourceResult(src.status, src.deliver_time_ns, src.event_id,
                           src.send if self.last_mode == "padded+exact" else None, send_counts, *self.last_stats,
                           send_padded=src.send_padded)
        self.last = (recv, order, offsets)
        self.last_recv_counts = list(recv_counts)
        return res, recv, recv_counts, order, offsets

    def _round_exact(self, packets, round_end_ns, sim_end_ns, bootstrap_end_ns):
        self.last_mode = "exact"
        src = self.source_fn(self.ctx, self.hosts, self.table, packets, round_end_ns, sim_end_ns, bootstrap_end_ns,
                             self.owner_dev, self.world)
        stats = (int(src.n_delivered), int(src.min_deliver_time_ns), int(src.min_used_latency_ns))
        self.last_send_counts = list(src.send_counts)
        if self.exchange_fn is None:
            recv, recv_counts, self.last_stats, self._pair_max = exchange_round(
                src.send, src.send_counts, stats, self.rank, self.dist, self.group, ws=self.ws, want_pair_max=True)
        else:
            recv, recv_counts = self.exchange_fn(src.send, src.send_counts)
            self.last_stats = gather_round_stats(*stats, self.dist, self.group, self.device)
            # the block size must agree on every rank: the largest pair count of all ranks
            self._pair_max = _global_max(max(list(src.send_counts) + list(recv_counts) + [0]), self.dist,
                                         self.group, self.device)
        order, offsets = self.bucket_fn(self.ctx, recv, int(sum(recv_counts)), self.local_dev,
                                        len(self.part.local), self.part.n_local(self.rank))
        self.last = (recv, order, offsets)  # this rank's destination buckets of the round
        self.last_recv_counts = list(recv_counts)
        return src, recv, recv_counts, order, offsets
