"""The sharded path's collectives through the C ABI (sg_comm_*, include/shadow_gpu.h, ABI 7).

One RCCL communicator per rank, bound to a Context: every exchange is enqueued on the
context's stream inside libshadow_gpu.so, so the Rust caller of INTEGRATION.md makes the
same calls this module does (no torch in the data path).  torch.distributed is used
here only to hand rank 0's unique id to the other ranks, as the reference's manager
would over its own channel.

    comm = Comm.from_torch(ctx, torch.distributed)     # or Comm(ctx, uid, n_ranks, rank)
    comm.allgather_rows(lat, loss, rows_per_rank, n_used)            # APSP row blocks
    recv, xall = comm.exchange_padded(send_padded, xrow, cap)       # fixed-split round exchange
    recv = comm.alltoallv_records(send, send_counts, recv_counts)    # exact exchange
"""
from __future__ import annotations

import ctypes as C
from typing import List, Optional

from . import _capi
from ._capi import check, load


def _ptr(t) -> int:
    return int(t.data_ptr()) if t is not None else 0


class Comm:
    """An sg_comm: RCCL over xGMI on the context's device and stream."""

    def __init__(self, ctx, uid: bytes, n_ranks: int, rank: int):
        if len(uid) != _capi.SG_COMM_ID_BYTES:
            raise ValueError("unique id must be SG_COMM_ID_BYTES long")
        L = load()
        h = C.c_void_p()
        buf = (C.c_uint8 * _capi.SG_COMM_ID_BYTES).from_buffer_copy(uid)
        check(ctx.handle, L.sg_comm_create(ctx.handle, C.addressof(buf), int(n_ranks), int(rank), C.byref(h)))
        self.handle, self.ctx, self.n_ranks, self.rank = h, ctx, int(n_ranks), int(rank)

    @staticmethod
    def unique_id() -> bytes:
        buf = (C.c_uint8 * _capi.SG_COMM_ID_BYTES)()
        rc = load().sg_comm_unique_id(C.addressof(buf))
        if rc != _capi.SG_OK:
            raise _capi.ShadowGpuError(rc, f"sg_comm_unique_id failed with status {rc}")
        return bytes(buf)

    @classmethod
    def from_torch(cls, ctx, dist, group=None) -> "Comm":
        """Rank 0 makes the id; torch.distributed broadcasts its bytes to the others.  Raises
        ShadowGpuError on every rank alike when RCCL cannot be set up on some rank (see
        _agree): no rank is left waiting in a collective the others never enter."""
        import torch

        rank, world = dist.get_rank(group), dist.get_world_size(group)
        dev = "cpu" if dist.get_backend(group) == "gloo" else torch.device("cuda", torch.cuda.current_device())
        # every rank opens RCCL first (sg_comm_unique_id also probes the library), and the
        # ranks agree on the outcome before any of them enters the communicator's setup
        uid, code = b"", _capi.SG_OK
        try:
            uid = cls.unique_id()
        except _capi.ShadowGpuError as e:
            code = e.code
        code = _agree(code, dist, group, dev)
        if code != _capi.SG_OK:
            raise _capi.ShadowGpuError(code, "sg_comm_unique_id failed on some rank")
        t = torch.zeros(_capi.SG_COMM_ID_BYTES, dtype=torch.uint8, device=dev)
        if rank == 0:
            t.copy_(torch.frombuffer(bytearray(uid), dtype=torch.uint8))
        if world > 1:
            dist.broadcast(t, 0, group=group)
        comm, code = None, _capi.SG_OK
        try:
            comm = cls(ctx, bytes(t.cpu().numpy().tobytes()), world, rank)
        except _capi.ShadowGpuError as e:
            code = e.code
        code = _agree(code, dist, group, dev)
        if code != _capi.SG_OK:
            if comm is not None:
                comm.close()
            raise _capi.ShadowGpuError(code, "sg_comm_create failed on some rank")
        return comm

    def get_world_size(self, group=None) -> int:
        return self.n_ranks

    def get_rank(self, group=None) -> int:
        return self.rank

    def close(self) -> None:
        if getattr(self, "handle", None):
            load().sg_comm_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # --- collectives (device tensors, the context's stream) -----------------------
    def allgather_rows(self, lat, loss, rows_per_rank: int, n_used: int) -> None:
        """In place: rank r's row block of the (n_ranks * rows_per_rank) x n_used table to every rank."""
        check(self.ctx.handle, load().sg_comm_allgather_rows(self.handle, _ptr(lat), _ptr(loss), int(rows_per_rank),
                                                              int(n_used)))

    def allgather_u64(self, mine, out) -> None:
        check(self.ctx.handle, load().sg_comm_allgather_u64(self.handle, _ptr(mine), _ptr(out), int(mine.numel())))

    def exchange_padded(self, send_padded, recv_padded, cap: int, xrow, xall) -> None:
        """xrow -> xall (all-gather) and cap records per rank pair send_padded -> recv_padded."""
        check(self.ctx.handle, load().sg_comm_exchange_padded(self.handle, _ptr(send_padded), _ptr(recv_padded),
                                                               int(cap), _ptr(xrow), _ptr(xall)))

    def alltoallv_records(self, send, send_counts: List[int], recv, recv_counts: List[int]) -> None:
        sc = (C.c_uint32 * self.n_ranks)(*[int(x) for x in send_counts])
        rc = (C.c_uint32 * self.n_ranks)(*[int(x) for x in recv_counts])
        check(self.ctx.handle, load().sg_comm_alltoallv_records(self.handle, _ptr(send), sc, _ptr(recv), rc))


def _agree(code: int, dist, group, dev) -> int:
    """The largest status over the ranks (status codes are >= 0, SG_OK = 0): one all-reduce, so
    every rank takes the same branch."""
    import torch

    if dist.get_world_size(group) <= 1:
        return int(code)
    t = torch.tensor([int(code)], dtype=torch.int64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return int(t.item())


def is_comm(d) -> bool:
    return isinstance(d, Comm)


def maybe_comm(ctx, dist, group=None) -> Optional[Comm]:
    """A Comm for an RCCL process group (None for gloo, or when RCCL cannot be opened on some
    rank: then on every rank, so all of them fall back to torch.distributed together)."""
    if dist is None or dist.get_backend(group) == "gloo":
        return None
    try:
        return Comm.from_torch(ctx, dist, group)
    except _capi.ShadowGpuError as e:
        if e.code == _capi.SG_ERR_UNSUPPORTED:
            return None
        raise
