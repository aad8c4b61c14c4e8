"""World-size-2 gloo tests of the sharding logic on CPU.

The exchange code (`shadow_amd.dist.all_to_all_records`, `ShardedDelivery`) and
the row partition are the real product code; the GPU phases are replaced by
numpy/oracle stand-ins written here (the kernels themselves are covered by
tests/test_dist_gpu.py on the GPU box).  The merged result must equal a single
oracle round over all packets, and gathered row shards the full table.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from shadow_amd import synth
from shadow_amd.dist import (HostPartition, RECORD_DTYPE, ShardedDelivery, SourcePadded, SourceResult,
                             balanced_node_order, row_range)

T0 = 946684800 * 10**9
NONE = 0xFFFFFFFF


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _world(O, skew=False, world=2):
    """skew: 200 nodes, 90 % of the hosts on 1 % of them (nodes 0 and 1, one routing-row
    block under the identity order), rows in balanced_node_order's order."""
    n = 200 if skew else 60
    g = synth.ring_chords_graph(n, 6.0, seed=2)
    hosts = synth.make_hosts(400, n, general_seed=4)
    used = np.arange(n, dtype=np.uint32)
    if skew:
        node = np.where(np.arange(400) % 10 < 9, np.arange(400) % 2, 2 + np.arange(400) % (n - 2)).astype(np.uint32)
        used, hosts["route"] = balanced_node_order(node, n, world)
        hosts["node"] = node
    rc, lat, loss, _ = O.shortest_paths(n, g["src"], g["dst"], g["lat"], g["loss"], False, used, threads=2)
    assert rc == 0
    loss = loss.copy()
    loss[::2, 1::2] = np.float32(0.35)
    pk = synth.make_packets(12000, hosts, T0, T0 + 10**6, seed=8, p_unknown_dst=0.02)
    return g, lat, loss, hosts, pk, used


class _Tables:
    """Stand-in for the device state of one rank (test-side only)."""

    def __init__(self, O, hosts):
        self.rng = np.stack([O.xoshiro_seed(int(s)) for s in hosts["seed"]]).astype(np.uint64)
        self.ctr = np.zeros(hosts["n"], np.uint64)


def _cpu_source(O, lat, loss, hosts, state, part):
    def fn(ctx, h, table, packets, round_end, sim_end, boot, owner_dev, n_ranks):
        src, dst_ip, pay, t = packets
        ctr0 = state.ctr.copy()
        res = O.deliver_round(round_end, sim_end, boot, src, dst_ip, pay, t, hosts["ip"], hosts["route"], lat, loss,
                              state.rng, state.ctr)
        ip2h = {int(ip): k for k, ip in enumerate(hosts["ip"])}
        recs = []
        for i in np.nonzero(res["status"] == O.ST_DELIVERED)[0]:
            s, d = int(src[i]), ip2h[int(dst_ip[i])]
            k = int(res["event_id"][i] - ctr0[s])
            recs.append((int(res["deliver_time"][i]), (s << 32) | k, int(res["event_id"][i]), int(i), d))
        recs = np.array(recs, dtype=RECORD_DTYPE) if recs else np.zeros(0, RECORD_DTYPE)
        own = part.owner[recs["dst_host"]]
        recs = recs[np.argsort(own, kind="stable")]
        counts = [int((own == r).sum()) for r in range(n_ranks)]
        send = torch.from_numpy(recs.view(np.int64).reshape(-1, 4).copy())
        return SourceResult(res["status"], res["deliver_time"], res["event_id"], send, counts, res["delivered"],
                            res["min_deliver"], res["min_lat"])
    return fn


def _cpu_bucket(part, rank):
    def fn(ctx, recv, n, local_dev, n_hosts, n_local):
        rec = recv.numpy().view(RECORD_DTYPE).ravel()[:n]
        slot = part.local[rec["dst_host"]]
        assert (part.owner[rec["dst_host"]] == rank).all()
        order = np.lexsort((rec["order_key"], rec["deliver_time_ns"], slot)).astype(np.uint32)
        offsets = np.zeros(n_local + 1, np.uint32)
        np.add.at(offsets, slot + 1, 1)
        return order, np.cumsum(offsets).astype(np.uint32)
    return fn


def _worker(rank, world, port, q, skew=False):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from oracle import oracle as O

        g, lat, loss, hosts, pk, used = _world(O, skew, world)
        nu = lat.shape[0]
        # --- routing rows: each rank its block, all-gathered ---
        r0, r1, per = row_range(nu, world, rank)
        rc, mine, _, _ = O.shortest_paths(g["n"], g["src"], g["dst"], g["lat"], g["loss"], False, used,
                                          rows=(r0, r1))
        block = np.zeros((per, nu), np.uint64)
        block[: r1 - r0] = mine
        full = torch.zeros(world * per * nu, dtype=torch.int64)
        dist.all_gather_into_tensor(full, torch.from_numpy(block.view(np.int64).ravel()))
        gathered = full.numpy().view(np.uint64).reshape(world * per, nu)[:nu]
        rows_ok = bool(np.array_equal(gathered, lat))
        # --- sharded delivery ---
        part = HostPartition(hosts["route"], nu, world)
        sel = np.nonzero(part.owner[pk["src"]] == rank)[0]
        state = _Tables(O, hosts)
        sd = ShardedDelivery(None, None, None, part, rank, world, dist=dist, device="cpu",
                             source_fn=_cpu_source(O, lat, loss, hosts, state, part),
                             bucket_fn=_cpu_bucket(part, rank))
        packets = (pk["src"][sel], pk["dst_ip"][sel], pk["payload"][sel], pk["send_time"][sel])
        src, recv, recv_counts, order, offsets = sd.round(packets, T0 + 10**6, 2**63, 0)
        rec = recv.numpy().view(RECORD_DTYPE).ravel()
        # map records back to global packet indices: sender r's selection
        sels = [np.nonzero(part.owner[pk["src"]] == r)[0] for r in range(world)]
        origin = np.repeat(np.arange(world), recv_counts)
        glob = np.array([sels[origin[k]][rec["packet"][k]] for k in range(len(rec))], np.int64)
        per_dst = {int(h): glob[order[offsets[s]:offsets[s + 1]]].tolist() for s, h in enumerate(part.hosts_of[rank])}
        q.put((rank, rows_ok, per_dst, src.status.tolist(), sel.tolist(), sd.last_stats))
        dist.destroy_process_group()
    except Exception as e:  # surface worker failures to the parent
        import traceback

        q.put((rank, "error", traceback.format_exc(), None, None, None))


@pytest.mark.parametrize("skew", [False, True])
def test_two_rank_gloo_exchange_matches_single_round(oracle, skew):
    """The sharded round equals one oracle round.  skew: 90 % of the hosts on 1 % of the
    nodes; with balanced_node_order's rows each rank sends within 1.5x of the other."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, skew)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for o in out:
        assert o[1] != "error", o[2]
    g, lat, loss, hosts, pk, used = _world(oracle, skew, world)
    if skew:
        sent = [len(o[4]) for o in out]
        assert max(sent) <= 1.5 * min(sent), sent
        # the identity row order would put both hot nodes, and ~94 % of the senders, on rank 0
        ident = HostPartition(hosts["node"], g["n"], world)
        assert (ident.owner[pk["src"]] == 0).mean() > 0.9
    rng = np.stack([oracle.xoshiro_seed(int(s)) for s in hosts["seed"]]).astype(np.uint64)
    ctr = np.zeros(hosts["n"], np.uint64)
    want = oracle.deliver_round(T0 + 10**6, 2**63, 0, pk["src"], pk["dst_ip"], pk["payload"], pk["send_time"],
                                hosts["ip"], hosts["route"], lat, loss, rng, ctr)
    seen = set()
    for rank, rows_ok, per_dst, status, sel, stats in out:
        assert rows_ok
        assert stats == (want["delivered"], want["min_deliver"], want["min_lat"])  # global round scalars
        assert np.array_equal(np.array(status, np.uint8), want["status"][np.array(sel, np.int64)])
        for h, got in per_dst.items():
            exp = want["dst_order"][want["dst_offsets"][h]:want["dst_offsets"][h + 1]].tolist()
            assert got == exp, h
            seen.add(h)
    assert seen == set(range(hosts["n"]))


# ---- the fixed-split exchange (ShardedDelivery(padded=True)) over gloo ---------------
def _cpu_source_padded(O, lat, loss, hosts, state, part):
    exact = _cpu_source(O, lat, loss, hosts, state, part)

    def fn(ctx, h, table, packets, round_end, sim_end, boot, owner_dev, n_ranks, cap):
        r = exact(ctx, h, table, packets, round_end, sim_end, boot, owner_dev, n_ranks)
        recs = r.send.numpy()
        padded = np.zeros((n_ranks * cap, 4), np.int64)
        send = np.zeros_like(recs)
        start = 0
        for d, c in enumerate(r.send_counts):
            k = min(c, cap)
            padded[d * cap:d * cap + k] = recs[start:start + k]
            send[start + k:start + c] = recs[start + k:start + c]  # past cap: compact positions only
            start += c
        xrow = np.array([r.n_delivered, r.min_deliver_time_ns, r.min_used_latency_ns, *r.send_counts],
                        np.uint64).view(np.int64)
        return SourcePadded(r.status, r.deliver_time_ns, r.event_id, torch.from_numpy(padded), torch.from_numpy(send),
                            torch.from_numpy(xrow.copy()), cap)
    return fn


def _cpu_bucket_padded(part, rank):
    def fn(ctx, recv, cap, xall, rk, local_dev, n_hosts, n_local):
        world = recv.shape[0] // cap
        xa = xall.numpy().view(np.uint64).reshape(world, 3 + world)
        rec = recv.numpy().view(RECORD_DTYPE).ravel()
        idx = np.concatenate([b * cap + np.arange(min(int(xa[b, 3 + rank]), cap)) for b in range(world)])
        idx = idx.astype(np.int64)
        slot = part.local[rec["dst_host"][idx]]
        assert (part.owner[rec["dst_host"][idx]] == rank).all()
        o = np.lexsort((rec["order_key"][idx], rec["deliver_time_ns"][idx], slot))
        offsets = np.zeros(n_local + 1, np.uint32)
        np.add.at(offsets, slot + 1, 1)
        stats = (int(xa[:, 0].sum()), int(xa[:, 1].min()), int(xa[:, 2].min()))
        return (idx[o].astype(np.uint32), np.cumsum(offsets).astype(np.uint32), stats,
                [int(x) for x in xa[:, 3 + rank]], int(xa[:, 3:].max()))
    return fn


def _cpu_pad_to_compact(ctx, src, n_ranks):
    xrow = src.xrow.numpy().view(np.uint64)
    send = src.send.numpy()
    pad = src.send_padded.numpy()
    start = 0
    for d in range(n_ranks):
        c = int(xrow[3 + d])
        k = min(c, src.cap)
        send[start:start + k] = pad[d * src.cap:d * src.cap + k]
        start += c
    return src.send


def _worker_padded(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from oracle import oracle as O

        g, lat, loss, hosts, _, used = _world(O, False, world)
        nu = lat.shape[0]
        part = HostPartition(hosts["route"], nu, world)
        state = _Tables(O, hosts)
        sd = ShardedDelivery(None, None, None, part, rank, world, dist=dist, device="cpu", padded=True,
                             source_fn=_cpu_source(O, lat, loss, hosts, state, part),
                             bucket_fn=_cpu_bucket(part, rank),
                             source_padded_fn=_cpu_source_padded(O, lat, loss, hosts, state, part),
                             bucket_padded_fn=_cpu_bucket_padded(part, rank), pad_to_compact_fn=_cpu_pad_to_compact)
        results = []
        for k in range(4):  # exact (sizes the blocks), padded, padded with a hot destination (overflow), padded
            start = T0 + k * 10**6
            hot = k == 2
            pk = synth.make_packets(12000, hosts, start, start + 10**6, seed=20 + k, p_unknown_dst=0.02,
                                    hot_dst=5 if hot else -1, p_hot=0.6 if hot else 0.0)
            sel = np.nonzero(part.owner[pk["src"]] == rank)[0]
            packets = (pk["src"][sel], pk["dst_ip"][sel], pk["payload"][sel], pk["send_time"][sel])
            src, recv, recv_counts, order, offsets = sd.round(packets, start + 10**6, 2**63, 0)
            rec = recv.numpy().view(RECORD_DTYPE).ravel()
            sels = [np.nonzero(part.owner[pk["src"]] == r)[0] for r in range(world)]
            if sd.last_mode == "padded":  # block b of cap records came from rank b
                origin = np.arange(len(rec)) // sd_cap_prev
            else:
                origin = np.repeat(np.arange(world), recv_counts)
            glob = {}
            for s_, hh in enumerate(part.hosts_of[rank]):
                ks = np.asarray(order[offsets[s_]:offsets[s_ + 1]], np.int64)
                glob[int(hh)] = [int(sels[origin[k_]][rec["packet"][k_]]) for k_ in ks]
            results.append((sd.last_mode, glob, np.asarray(src.status).tolist(), sel.tolist(), sd.last_stats))
            sd_cap_prev = sd.cap  # the block size the next round uses
        q.put((rank, results))
        dist.destroy_process_group()
    except Exception:
        import traceback

        q.put((rank, "error", traceback.format_exc()))


def test_two_rank_gloo_padded_exchange_rounds(oracle):
    """ShardedDelivery(padded=True) over gloo: the first round is exact and sizes the
    blocks, the next ones use the fixed-split exchange (no host round trip before the
    round's end); a round whose hot destination overfills a block is exchanged again
    exactly.  Every round equals one oracle round over all packets."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_padded, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for o in out:
        assert o[1] != "error", o[2]
    g, lat, loss, hosts, _, used = _world(oracle, False, world)
    rng = np.stack([oracle.xoshiro_seed(int(s)) for s in hosts["seed"]]).astype(np.uint64)
    ctr = np.zeros(hosts["n"], np.uint64)
    modes = []
    for k in range(4):
        start = T0 + k * 10**6
        hot = k == 2
        pk = synth.make_packets(12000, hosts, start, start + 10**6, seed=20 + k, p_unknown_dst=0.02,
                                hot_dst=5 if hot else -1, p_hot=0.6 if hot else 0.0)
        want = oracle.deliver_round(start + 10**6, 2**63, 0, pk["src"], pk["dst_ip"], pk["payload"], pk["send_time"],
                                    hosts["ip"], hosts["route"], lat, loss, rng, ctr)
        seen = set()
        for rank, results in out:
            mode, per_dst, status, sel, stats = results[k]
            modes.append(mode)
            assert stats == (want["delivered"], want["min_deliver"], want["min_lat"]), (k, mode)
            assert np.array_equal(np.array(status, np.uint8), want["status"][np.array(sel, np.int64)])
            for h, got in per_dst.items():
                assert got == want["dst_order"][want["dst_offsets"][h]:want["dst_offsets"][h + 1]].tolist(), (k, h)
                seen.add(h)
        assert seen == set(range(hosts["n"]))
    assert modes == ["exact"] * 2 + ["padded"] * 2 + ["padded+exact"] * 2 + ["padded"] * 2, modes


def test_balanced_order_keeps_local_blocks():
    """A host map the identity order already balances keeps it (row blocks stay runs of
    consecutive nodes, whose neighbours bound the blocks' searches); a skewed one is
    dealt by weight, each rank within one node's weight of the mean."""
    order, route = balanced_node_order(np.arange(100_000) % 10_000, 10_000, 8)
    assert np.array_equal(order, np.arange(10_000)) and np.array_equal(route, np.arange(100_000) % 10_000)
    node = np.where(np.arange(4000) % 10 < 9, np.arange(4000) % 2, 2 + np.arange(4000) % 198)
    order, route = balanced_node_order(node, 200, 2)
    assert not np.array_equal(order, np.arange(200))
    pos = np.empty(200, np.int64)
    pos[order] = np.arange(200)
    load = np.bincount(pos[node] // 100, minlength=2)
    w = np.bincount(node, minlength=200)
    assert abs(int(load[0]) - int(load[1])) <= w.max()
    assert np.array_equal(route, pos[node])


def _agree_worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from shadow_amd import _capi
        from shadow_amd import comm as CM

        got = [CM._agree(_capi.SG_OK, dist, None, "cpu"),
               CM._agree(_capi.SG_ERR_UNSUPPORTED if rank == 1 else _capi.SG_OK, dist, None, "cpu")]

        # sg_comm_unique_id failing on rank 1 only: every rank raises the same status, none
        # enters the broadcast or the communicator's setup alone
        def uid():
            if rank == 1:
                raise _capi.ShadowGpuError(_capi.SG_ERR_UNSUPPORTED, "no RCCL here")
            return bytes(_capi.SG_COMM_ID_BYTES)

        CM.Comm.unique_id = staticmethod(uid)
        try:
            CM.Comm.from_torch(None, dist)
            got.append(None)
        except _capi.ShadowGpuError as e:
            got.append(e.code)
        dist.destroy_process_group()
        q.put((rank, got))
    except Exception:
        import traceback

        q.put((rank, traceback.format_exc()))


def test_comm_setup_agrees_across_ranks():
    """comm.Comm.from_torch / maybe_comm: a failure on one rank is every rank's failure."""
    from shadow_amd import _capi

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_agree_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for rank, got in out:
        assert got == [_capi.SG_OK, _capi.SG_ERR_UNSUPPORTED, _capi.SG_ERR_UNSUPPORTED], (rank, got)
