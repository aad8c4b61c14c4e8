#!/usr/bin/env python3
"""Benchmark of the MI355X network core against BASELINE.json's metric:

  "APSP routing build (s) @10k nodes; packets routed/sec per sim round"

Primary line (`value`): one routing-table build of the C3 workload (10k-node
ring + chords, mean degree 8, every node used) -- seconds per
build, source rows sharded across ranks (rows are independent units; each rank
keeps its row block, which is all delivery reads).  The optional RCCL all-gather
that would replicate the table is timed separately (apsp_detail.allgather_ms).
`delivery` sub-object: one C4 delivery round (100k hosts, 1M packets per rank)
per step, packets/s; at N > 1 delivered records go to the destination's owner
by RCCL all-to-all.  Inputs are resident in HBM when the timed region starts.

Single GPU:  python bench.py [--steps K --warmup W]
N GPUs:      python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "APSP routing build (s) @10k nodes; packets routed/sec per sim round"
# Peaks (/opt/skills/guides/MI355X_MICROARCH.md, chip-level table)
HBM_PEAK_GBS = 8000.0
# 157.3 TFLOP/s FP32 vector = 256 CU x 4 SIMD x 32 lanes x 2.4 GHz x 2 (FMA) -> 78.6 T 32-bit VALU ops/s
VALU_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12
# L2: 4 MiB per XCD, ~34.5 TB/s aggregate (MI355X_MICROARCH.md, "L2 (per XCD)")
L2_PEAK_GBS = 34500.0
ROW_BYTES_PER_RELAX = 8  # slab kernel: one 8-B packed key gathered per lane-relaxation (512-B row per 64 sources)
ARC_BYTES_PER_RELAX = 12  # LDS search: one 12-B out-arc record (head, latency, 1 - loss) read per relaxation
FAITHFUL_ROWS = 400  # sources in the reference-faithful CPU sample (~10 s of CPU work at C3 on 16 threads)
C5_CPU_ROWS = 1024  # C5 dense-port sample (the first rows, scaled by 50k / 1,024)
C5_FAITHFUL_ROWS = 96  # C5 reference-faithful sample (~5x C3's cost per source)


def _cpu_info():
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    visible = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    # the CPU share this process may use: the GPU box grants 16 logical CPUs per GPU (a
    # quota, while all of the host's CPUs stay visible) and says so in OMP_NUM_THREADS
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or visible
    return {"nproc": min(share, visible), "nproc_visible": visible, "cpu_model": model}


CPU_INFO = _cpu_info()
# the reference's pools: rayon's global pool for APSP = all logical CPUs; the worker
# threads = the physical cores (manager.rs:254-261).  Both are the CPU share here:
# more threads than the share only time-slice on it (r02: 256 threads on the 16-CPU
# share took 1.55 s for the dense C3 baseline, 16 threads 1.17 s).
CPU_THREADS = CPU_INFO["nproc"]
T0 = 946684800 * 10**9  # EmulatedTime SIMULATION_START


PMC_DEFAULT = os.path.join(ROOT, "profiles", "pmc_latest.json")
PMC_C5 = os.path.join(ROOT, "profiles", "pmc_c5_latest.json")


def parse_args():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--nodes", type=int, default=10000)
    p.add_argument("--degree", type=float, default=8.0)
    p.add_argument("--hosts", type=int, default=100000)
    p.add_argument("--packets", type=int, default=1000000)
    p.add_argument("--config", choices=("c3c4", "c5"), default="c3c4",
                   help="c3c4 (default): the C3 routing build + C4 delivery round (weak scaling, 1M packets per "
                        "rank); c5: SURVEY 8d C5, a 50k-node graph and 10M packets per round in total, split "
                        "over the ranks (strong scaling)")
    p.add_argument("--cpu-rows", type=int, default=None,
                   help="time the CPU routing baseline on the first K source rows and scale to all rows "
                        "(0 = every row; default: every row at C3, the first 1,024 at C5)")
    p.add_argument("--rank-blocks", default="2,4,8",
                   help="at one GPU: time every rank's one-shot row-block build of these N-way splits "
                        "(apsp_detail.rank_block_ms; '' skips)")
    p.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    p.add_argument("--no-delivery", action="store_true")
    p.add_argument("--no-e2e", action="store_true",
                   help="skip the end-to-end RoutingInfo fill (its row-block launches of the search would mix "
                        "into a profile of the headline's whole-table launches)")
    p.add_argument("--no-codel", action="store_true", help="skip the router CoDel leg")
    p.add_argument("--no-gml", action="store_true", help="skip the GML ingest leg")
    p.add_argument("--no-c2", action="store_true", help="skip the C2 (1,200-node complete graph) leg")
    p.add_argument("--no-compare", action="store_true",
                   help="skip the comparison builds (slab kernel, one-launch unbounded search): for rocprof "
                        "runs whose k_sssp_lds average must be the default plan's alone")
    p.add_argument("--exact-exchange", action="store_true",
                   help="N > 1: exchange every round's records with host-sized splits (one host round trip "
                        "more per round) instead of the fixed-split exchange")
    p.add_argument("--no-pack", action="store_true",
                   help="deliver from the two-array table (no packed path-key copy)")
    p.add_argument("--pmc-json", default=PMC_DEFAULT,
                   help="PMC summary (HBM bytes per launch) written by tools/pmc_summary.py (C5: "
                        "profiles/pmc_c5_latest.json)")
    a = p.parse_args()
    if a.config == "c5":
        a.nodes, a.hosts, a.packets = 50000, 100000, 10000000
    if a.cpu_rows is None:  # C5: ~25x C3's CPU work per row; a sample of ~20-30 s on the 16-CPU share
        a.cpu_rows = C5_CPU_ROWS if a.config == "c5" else 0
    return a


class Dist:
    def __init__(self, n_gpus):
        import torch

        self.torch = torch
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        if self.world != n_gpus:
            raise SystemExit(f"--gpus {n_gpus} but WORLD_SIZE={self.world}")
        # more ranks than GPUs (a rehearsal of the N-rank path on a smaller box) share devices
        self.local %= max(1, torch.cuda.device_count())
        torch.cuda.set_device(self.local)
        self.dist = None
        if self.world > 1:
            import torch.distributed as dist

            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            # SG_BENCH_BACKEND=gloo: rehearse the N-rank path with more ranks than GPUs
            # (RCCL refuses two ranks on one device); collectives are host-staged, so its
            # timings are not measurements
            self.backend = os.environ.get("SG_BENCH_BACKEND", "nccl")
            if self.backend == "gloo":
                dist.init_process_group("gloo")
            else:
                dist.init_process_group("nccl", device_id=torch.device("cuda", self.local))
            self.dist = dist
        self.coll_dev = "cpu" if self.dist and self.backend == "gloo" else "cuda"

    def barrier(self):
        if self.dist:
            self.dist.barrier()

    def max(self, x: float) -> float:
        if not self.dist:
            return x
        t = self.torch.tensor([x], dtype=self.torch.float64, device=self.coll_dev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def gather(self, xs):
        """Every rank's list of floats (rank order)."""
        if not self.dist:
            return [list(xs)]
        t = self.torch.tensor(list(xs), dtype=self.torch.float64, device=self.coll_dev)
        out = self.torch.empty(self.world * len(xs), dtype=self.torch.float64, device=self.coll_dev)
        self.dist.all_gather_into_tensor(out, t)
        return out.cpu().view(self.world, len(xs)).tolist()

    def sum(self, x: float) -> float:
        if not self.dist:
            return x
        t = self.torch.tensor([x], dtype=self.torch.float64, device=self.coll_dev)
        self.dist.all_reduce(t)
        return float(t.item())


_T_START = time.perf_counter()


def note(msg: str) -> None:
    """A progress line on stderr (a long run stays visibly alive; stdout keeps the one JSON line)."""
    print(f"[bench {time.perf_counter() - _T_START:7.1f} s] {msg}", file=sys.stderr, flush=True)


def timed(D, fn, steps, warmup):
    torch = D.torch
    for _ in range(warmup):
        fn()
    D.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    D.barrier()
    return D.max(time.perf_counter() - t0) / steps


def _pow2(x):
    return 1 << max(0, int(x) - 1).bit_length()


def queue_ahead(ctx, torch, cycles=2_000_000):
    """Hold the library's stream in a ~1 ms spin kernel, so that the launches (and HIP-event
    markers) the host enqueues next are already queued when the GPU reaches them.  An event
    pair then brackets its kernel plus the ~1 us between back-to-back dispatches; enqueued on
    an idle stream it also held the host's launch latency (~10 us against a 30-50 us lane
    kernel, r04t: k_codel 49 us by events against 34.6 us in the rocprof trace)."""
    s = torch.cuda.ExternalStream(ctx.stream) if ctx.stream else torch.cuda.current_stream()
    with torch.cuda.stream(s):
        torch.cuda._sleep(cycles)


# The lane kernels' HIP-event pairs: queue_ahead keeps the host ahead of the GPU, and each pair still
# holds the command processor's gap between the kernel before and the one it brackets (~4-5 us
# against 30-50 us kernels: r6, tools/inbound_timer_diag.py, profiles/r06/ab_lane_timers_r6.txt);
# the line's "rocprof" object beside it gives the kernel-trace duration of the same kernel.  (A
# kernel launched with hipExtLaunchKernelGGL's own events measured the same gap; the kernel's span
# from its first block's start to its last block's end, by the device wall clock, fell 1-4 us
# short of rocprof's: neither is used.)
EVENT_TIMER = "HIP event pair around the launch (holds a ~4-5 us dispatch gap; rocprof beside it)"


def rocprof_view(pm, bytes_per_launch):
    """The rocprofv3 kernel-trace average of a kernel (from the PMC summary of the default
    workload) and the HBM fraction it gives, beside the line's own HIP-event figure."""
    ns = pm.get("avg_ns")
    if not ns or not bytes_per_launch:
        return None
    return {"avg_launch_ms": round(ns / 1e6, 4),
            "frac": round(bytes_per_launch / (ns / 1e9) / 1e9 / HBM_PEAK_GBS, 4)}


def load_pmc(path):
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return {}


SERVICE_NS = 12_000  # 1500 B at 1 Gbit/s: the interface's pop spacing in the CoDel leg
TIMED_REPS = 10  # HIP-event timed runs of the CoDel batch (its roofline)
SUB_MS_REPS = 100  # timed repetitions of the sub-millisecond legs (delivery round, CoDel batch) at least


def codel_events(offsets, order, deliver_time, length):
    """C4 round -> each destination's inbound CoDel stream: pushes at the arrival
    times (the bucket, in EventQueue order) and a FIFO server popping one packet
    every SERVICE_NS (s_j = max(a_j, s_{j-1}) + SERVICE_NS); per host in time order,
    a push before a pop at the same time."""
    H = len(offsets) - 1
    cnt = np.diff(offsets.astype(np.int64))
    host = np.repeat(np.arange(H, dtype=np.int64), cnt)
    arr = deliver_time[order].astype(np.int64)
    j = np.arange(len(order), dtype=np.int64) - np.repeat(offsets[:-1].astype(np.int64), cnt)  # rank in bucket
    # s_j = (j + 1) S + max_{k<=j} (a_k - k S), a running max restarted per host: a per-host
    # offset above the key range keeps earlier hosts below later ones
    key = arr - j * SERVICE_NS
    kmin = int(key.min()) if len(key) else 0
    shift = host << 41
    run = np.maximum.accumulate(key - kmin + shift) - shift + kmin if len(key) else key
    pop_t = run + (j + 1) * SERVICE_NS
    n = len(order)
    ev_host = np.concatenate([host, host])
    ev_time = np.concatenate([arr, pop_t])
    ev_kind = np.concatenate([np.zeros(n, np.uint8), np.ones(n, np.uint8)])
    ev_pkt = np.concatenate([order.astype(np.int64), np.zeros(n, np.int64)])
    ln = length[order].astype(np.int64)
    ev_len = np.concatenate([ln, np.zeros(n, np.int64)])
    idx = np.lexsort((ev_kind, ev_time, ev_host))
    return (ev_host[idx].astype(np.uint32), ev_kind[idx], ev_time[idx].astype(np.uint64),
            ev_pkt[idx].astype(np.uint32), ev_len[idx].astype(np.uint32))


def round_buckets(out, payload, sharded):
    """This rank's destination buckets of the last round: (offsets, order, deliver time
    and packet length per order index).  Sharded: the received records; their payload
    is not exchanged, so every length is a full 1476-B data packet."""
    if sharded is None:
        nd = int(out.n_delivered)
        return (out.dst_offsets.cpu().numpy().view(np.uint32), out.dst_order[:nd].cpu().numpy().view(np.uint32),
                out.deliver_time_ns.cpu().numpy().view(np.uint64),
                (28 + np.asarray(payload, np.int64)).astype(np.uint32))  # IPv4 + UDP headers (packet.rs:388-390)
    recv, order, offsets = sharded.last
    rec = recv.cpu().numpy().view(np.uint64).reshape(-1, 4) if recv.shape[0] else np.zeros((0, 4), np.uint64)
    order = np.asarray(order.cpu().numpy() if hasattr(order, "cpu") else order).view(np.uint32)
    offsets = np.asarray(offsets.cpu().numpy() if hasattr(offsets, "cpu") else offsets).view(np.uint32)
    return offsets, order, rec[:, 0].copy(), np.full(len(rec), 1476, np.uint32)


def codel_leg(a, D, ctx, torch, buckets, n_packets, pmc):
    from shadow_amd.router import CoDelEvents, CoDelQueues

    offs, order, dtime, lens = buckets
    nd = len(order)
    n_packets = max(n_packets, len(dtime))
    evs = codel_events(offs, order, dtime, lens)
    E = len(evs[0])
    H = len(offs) - 1
    q = CoDelQueues(H, max(256, _pow2(int(np.diff(offs).max(initial=0)))), ctx=ctx)
    ev = CoDelEvents.from_numpy(*evs)
    status = torch.zeros(max(n_packets, 1), dtype=torch.uint8, device="cuda")
    state0 = q.get_state()

    def step():
        q.run(ev, status)

    t = timed(D, step, max(a.steps, SUB_MS_REPS), a.warmup)
    q.set_state(state0)
    ctx.enable_timers(True)
    for _ in range(TIMED_REPS):  # the same batch from the same state, each run queued behind a spin kernel
        q.set_state(state0)
        queue_ahead(ctx, torch)
        _, n_drop = q.run(ev, status)
    k_ms, k_n, k_bytes = ctx.read_timer("codel")
    ctx.enable_timers(False)
    k_s = k_ms / 1e3 / max(k_n, 1)
    ach = k_bytes / max(k_n, 1) / k_s / 1e9 if k_n else 0.0
    pm = pmc.get("codel", {})
    leg = {
        "metric": "CoDel queue operations/sec (router inbound, one queue per host)", "unit": "ops/s",
        "value": round(D.sum(float(E)) / t, 1), "higher_is_better": True, "ms_per_batch": round(t * 1e3, 4),
        "scaling": "weak", "dtype": "u64+f64",
        "config": {"workload": "the C4 round's delivered packets pushed into their destinations' CoDel queues at "
                               "arrival, each interface popping one packet per 12 us (1500 B at 1 Gbit/s)",
                   "hosts": H, "events": E, "pushes": nd},
        "roofline": {"kernel": "k_codel", "bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": pm.get("hbm_bytes_per_launch"),
                     "avg_launch_ms": round(k_s * 1e3, 4), "timer": EVENT_TIMER, "valu_frac_pmc": pm.get("valu_frac"),
                     "rocprof": rocprof_view(pm, k_bytes / max(k_n, 1))},
        "dropped": n_drop,
    }
    if D.rank == 0 and D.world == 1 and not a.no_cpu:
        from oracle import oracle as O

        def run(th):
            st = O.codel_state(H, q.cap)
            ost = np.zeros(max(n_packets, 1), np.uint8)
            t0 = time.perf_counter()
            O.codel_run(st, *evs, ost, threads=th)
            return time.perf_counter() - t0

        tc, tc1 = run(CPU_THREADS), run(1)
        leg["cpu_baseline"] = {"value": round(E / tc, 1), "unit": "ops/s", "cores": CPU_THREADS, "kind": "port",
                               **CPU_INFO, "single_thread": {"value": round(E / tc1, 1)},
                               "sample": f"the same {E} events through the C restatement of codel_queue.rs, hosts "
                                         f"round-robin over {CPU_THREADS} threads (thread_per_core.rs:62-64)"}
    return leg


BW_DOWN_BITS = 10**9  # every host's bandwidth down in the inbound leg


BW_UP_BITS = 10**9  # every host's bandwidth up in the outbound leg
HDR_BYTES = 40      # IPv4 + TCP headers: PacketRc::len() = payload + headers


def outbound_leg(a, D, ctx, torch, pk, hosts, ht, table, round_end, sharded, pmc):
    """The C4 round's sends through every source's outbound pipeline: interface fifo ->
    relay_inet_out token bucket (1 Gbit/s up) -> router -> send_packet, one window holding
    the round; and the fused round (outbound + delivery of the sent batch)."""
    from shadow_amd.router import OutboundPipeline
    from shadow_amd.worker import Deliveries, deliver_round

    n, H = len(pk["src"]), hosts["n"]
    ln = (pk["payload"] + HDR_BYTES).astype(np.uint32)
    pkt = np.arange(n, dtype=np.uint32)
    dev = lambda x, dt, tv: torch.from_numpy(np.ascontiguousarray(x, dtype=dt).view(tv)).cuda()
    args = (dev(pk["src"], np.uint32, np.int32), dev(pk["send_time"], np.uint64, np.int64),
            dev(pkt, np.uint32, np.int32), dev(ln, np.uint32, np.int32), dev(pk["payload"], np.uint32, np.int32),
            dev(pk["dst_ip"], np.uint32, np.int32))
    fwd = torch.full((max(n, 1),), -1, dtype=torch.int64, device="cuda")
    status = torch.zeros(max(n, 1), dtype=torch.uint8, device="cuda")
    bw = np.full(H, BW_UP_BITS, np.uint64)
    n_pipes = 2 * (a.steps + a.warmup) + 1
    cap = max(64, _pow2(int(np.bincount(pk["src"], minlength=H).max(initial=0))))  # deepest interface queue
    pipes = [OutboundPipeline(hosts["ip"], bw, cap, ctx=ctx) for _ in range(n_pipes)]  # a fresh state per step
    for p in pipes:
        p.sent_buffers(n + 4 * H, "cuda")
    it = iter(pipes)

    def step():
        return next(it).run(*args, round_end, 0, 2**63, fwd, status)

    t_step = timed(D, step, a.steps, a.warmup)
    out = Deliveries.allocate(n, H)

    def fused():
        batch, _ = step()
        if sharded:
            sharded.round(batch, round_end, 2**63, 0)
        else:
            deliver_round(ht, table, batch, round_end, 2**63, 0, out=out, ctx=ctx)

    t_fused = timed(D, fused, a.steps, a.warmup)
    ctx.enable_timers(True)
    queue_ahead(ctx, torch)
    batch, _ = step()
    k_ms, k_n, k_bytes = ctx.read_timer("outbound")
    c_ms, c_n, _ = ctx.read_timer("out_compact")
    ctx.enable_timers(False)
    k_s = k_ms / 1e3 / max(k_n, 1)
    ach = k_bytes / max(k_n, 1) / k_s / 1e9 if k_n else 0.0
    leg = {
        "metric": "outbound sends/sec (interface fifo -> relay token bucket -> send_packet batch, per host)",
        "unit": "sends/s", "value": round(D.sum(float(n)) / t_step, 1), "higher_is_better": True,
        "ms_per_window": round(t_step * 1e3, 4), "scaling": "weak", "dtype": "u64",
        "config": {"workload": "the C4 round's sends (per source host in send order, len = payload + 40 B) through "
                               "each host's interface and a 1 Gbit/s relay_inet_out token bucket, one window holding "
                               "the round", "hosts": H, "sends_per_rank": n, "bw_up_bits": BW_UP_BITS},
        "roofline": {"kernel": "k_outbound", "bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                     "traffic": pmc.get("outbound", {}).get("hbm_bytes_per_launch"),
                     "avg_launch_ms": round(k_s * 1e3, 4), "timer": EVENT_TIMER, "valu_frac_pmc": pmc.get("outbound", {}).get("valu_frac"),
                     "rocprof": rocprof_view(pmc.get("outbound", {}), k_bytes / max(k_n, 1))},
        "compact_ms": round(c_ms / max(c_n, 1), 4),
        "sent": len(batch),
        "fused_round": {"ms": round(t_fused * 1e3, 4), "packets_per_s": round(D.sum(float(n)) / t_fused, 1),
                        "what": "outbound window + delivery round of the sent batch"},
    }
    if D.rank == 0 and D.world == 1 and not a.no_cpu:
        from oracle import oracle as O

        def run(th):
            st = O.outbound_state(hosts["ip"], bw, pipes[0].cap)
            ctr = np.zeros(H, np.uint64)
            ofwd = np.full(max(n, 1), np.uint64(2**64 - 1))
            ost = np.zeros(max(n, 1), np.uint8)
            t0 = time.perf_counter()
            O.outbound_run(st, pk["src"], pk["send_time"], pkt, ln, pk["payload"], pk["dst_ip"], round_end, 0, 2**63,
                           ctr, ofwd, ost, threads=th)
            return time.perf_counter() - t0

        tc, tc1 = run(CPU_THREADS), run(1)
        leg["cpu_baseline"] = {"value": round(n / tc, 1), "unit": "sends/s", "cores": CPU_THREADS, "kind": "port",
                               **CPU_INFO, "single_thread": {"value": round(n / tc1, 1)},
                               "sample": f"the same {n} sends through the C restatement (interface fifo + "
                                         f"relay/mod.rs + token_bucket.rs), hosts round-robin over {CPU_THREADS} "
                                         "threads (thread_per_core.rs:62-64)"}
    return leg


def inbound_leg(a, D, ctx, torch, buckets, n_packets, pmc, round_end):
    """The C4 round's buckets through every destination's inbound pipeline: router
    CoDel queue -> relay_inet_in token bucket (1 Gbit/s down), one window that holds
    every arrival.  Timed through sg_inbound_run_ordered (each arrival's fate at its
    arrival index, a host's outputs consecutive); the by-packet-id call beside it."""
    from shadow_amd.router import InboundPipeline

    offs, order, dtime, lens = buckets
    offs = offs.astype(np.int64)
    nd = len(order)
    n_packets = max(n_packets, len(dtime))
    H = len(offs) - 1
    host = np.repeat(np.arange(H, dtype=np.uint32), np.diff(offs))
    t = dtime[order]
    ln = lens[order].astype(np.uint32)
    window_end = int(t.max()) + 1 if nd else round_end + 1
    dev = lambda x, dt, tv: torch.from_numpy(np.ascontiguousarray(x, dtype=dt).view(tv)).cuda()
    args = (dev(host, np.uint32, np.int32), dev(t, np.uint64, np.int64), dev(order, np.uint32, np.int32),
            dev(ln, np.uint32, np.int32))
    fwd = torch.full((max(n_packets, 1),), -1, dtype=torch.int64, device="cuda")
    status = torch.zeros(max(n_packets, 1), dtype=torch.uint8, device="cuda")
    bw = np.full(H, BW_DOWN_BITS, np.uint64)
    cap = max(256, _pow2(int(np.diff(offs).max(initial=0))))  # the deepest router queue
    pipes = [InboundPipeline(bw, cap, ctx=ctx) for _ in range(a.steps + a.warmup + 1)]  # a fresh state per step
    it = iter(pipes)
    a_fwd = torch.full((max(nd, 1),), -1, dtype=torch.int64, device="cuda")
    a_st = torch.zeros(max(nd, 1), dtype=torch.uint8, device="cuda")

    def step():
        next(it).run_ordered(*args, window_end, 0, 2**63, fwd, status, a_fwd, a_st)

    t_step = timed(D, step, a.steps, a.warmup)
    # (zeroed before the spin: this process's first fill kernel loads its code object on the host,
    # ~1 ms, and queued after the spin it left the GPU idle between the ops the timer brackets --
    # 17-us gaps, the r05 line's 0.0595 ms against 0.0414 ms by rocprof)
    a_st.zero_()
    torch.cuda.synchronize()
    ctx.enable_timers(True)
    queue_ahead(ctx, torch)
    n_drop = next(it).run_ordered(*args, window_end, 0, 2**63, fwd, status, a_fwd, a_st)
    k_ms, k_n, k_bytes = ctx.read_timer("inbound")
    ctx.enable_timers(False)
    k_s = k_ms / 1e3 / max(k_n, 1)
    ach = k_bytes / max(k_n, 1) / k_s / 1e9 if k_n else 0.0
    # the fates by packet id (one fresh window: every packet arrived in it)
    if nd:
        status[args[2].long()] = a_st[:nd]
    n_fwd = int((status.cpu().numpy() == 1).sum())
    # the by-packet-id call (sg_inbound_run) on the same window, for comparison
    pipes_id = [InboundPipeline(bw, cap, ctx=ctx) for _ in range(a.steps + a.warmup)]
    it_id = iter(pipes_id)
    fwd_id = torch.full((max(n_packets, 1),), -1, dtype=torch.int64, device="cuda")
    st_id = torch.zeros(max(n_packets, 1), dtype=torch.uint8, device="cuda")
    t_id = timed(D, lambda: next(it_id).run(*args, window_end, 0, 2**63, fwd_id, st_id), a.steps, a.warmup)
    del pipes_id
    leg = {
        "metric": "inbound arrivals/sec (router CoDel queue -> relay token bucket, per host)", "unit": "arrivals/s",
        "value": round(D.sum(float(nd)) / t_step, 1), "higher_is_better": True, "ms_per_window": round(t_step * 1e3, 4),
        "scaling": "weak", "dtype": "u64+f64",
        "config": {"workload": "the C4 round's delivered packets arriving at their destinations (EventQueue order) "
                               "through each host's router CoDel queue and a 1 Gbit/s relay_inet_in token bucket, "
                               "one window holding every arrival", "hosts": H, "arrivals": nd,
                   "bw_down_bits": BW_DOWN_BITS},
        "roofline": {"kernel": "k_inbound", "bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                     "traffic": pmc.get("inbound", {}).get("hbm_bytes_per_launch"), "avg_launch_ms": round(k_s * 1e3, 4),
                     "timer": EVENT_TIMER,
                     "valu_frac_pmc": pmc.get("inbound", {}).get("valu_frac"),
                     "rocprof": rocprof_view(pmc.get("inbound", {}), k_bytes / max(k_n, 1))},
        "forwarded": n_fwd, "dropped": n_drop,
        "by_packet_id": {"ms_per_window": round(t_id * 1e3, 4),
                         "same_fates": bool(torch.equal(st_id, status)),
                         "what": "sg_inbound_run: fates written at the packet id (scattered)"},
    }
    if D.rank == 0 and D.world == 1 and not a.no_cpu:
        from oracle import oracle as O

        def run(th):
            st = O.inbound_state(bw, cap)
            ctr = np.zeros(H, np.uint64)
            ofwd = np.full(max(n_packets, 1), np.uint64(2**64 - 1))
            ost = np.zeros(max(n_packets, 1), np.uint8)
            t0 = time.perf_counter()
            O.inbound_run(st, host, t, order, ln, window_end, 0, 2**63, ctr, ofwd, ost, threads=th)
            return time.perf_counter() - t0, ost

        (tc, ost), (tc1, _) = run(CPU_THREADS), run(1)
        leg["cpu_baseline"] = {"value": round(nd / tc, 1), "unit": "arrivals/s", "cores": CPU_THREADS, "kind": "port",
                               **CPU_INFO, "single_thread": {"value": round(nd / tc1, 1)},
                               "sample": f"the same {nd} arrivals through the C restatement (codel_queue.rs + "
                                         f"relay/mod.rs + token_bucket.rs), hosts round-robin over {CPU_THREADS} "
                                         "threads (thread_per_core.rs:62-64)"}
        leg["parity_vs_cpu"] = bool(np.array_equal(ost, status.cpu().numpy()))
    return leg


GML_NODES = 50000  # 10k-50k-node graphs


def gml_leg(a, NetworkGraph, synth):
    """GML ingest (NetworkGraph::parse, graph/mod.rs:134-181) of a 50k-node graph: the
    host C++ parser on the box's CPU share, and on one thread."""
    g = synth.ring_chords_graph(GML_NODES, a.degree, seed=1)
    raw = synth.graph_to_gml(g).encode()
    th = min(16, os.cpu_count() or 1)

    def best(threads, reps=3):
        t = []
        for _ in range(reps):
            t0 = time.perf_counter()
            p = NetworkGraph.parse(raw, threads=threads)
            t.append(time.perf_counter() - t0)
        assert p.n_nodes == g["n"] and np.array_equal(p.edge_latency_ns, g["lat"])
        return min(t)

    t_many, t_one = best(th), best(1)
    mb = len(raw) / 1e6
    return {"metric": "GML ingest MB/s (parse + edge conversion + id lookup)", "unit": "MB/s",
            "value": round(mb / t_many, 1), "higher_is_better": True, "ms": round(t_many * 1e3, 2), "threads": th,
            "single_thread": {"value": round(mb / t_one, 1), "ms": round(t_one * 1e3, 2)},
            "config": {"workload": f"{GML_NODES}-node ring+chords GML (synth.graph_to_gml), mean degree {a.degree}",
                       "bytes": len(raw), "nodes": int(g["n"]), "edges": int(len(g["src"]))}}


C2_NODES = 1200  # Tor-style complete graph, use_shortest_path: true


def c2_leg(a, ctx, torch, NetworkGraph, synth, with_cpu, pmc=None):
    """C2 (BASELINE configs[1]): a 1,200-node complete undirected GML graph (about 720k
    edges), every node used -- GML parse on the host, then the routing-table build on
    one GPU (shortest paths; the direct-path table beside it).  CPU baseline: the oracle's
    Dijkstra on the box's CPU share; its rows double as a parity check of the GPU table."""
    g = synth.complete_graph(C2_NODES, seed=1)
    raw = synth.graph_to_gml(g).encode()
    t0 = time.perf_counter()
    net = NetworkGraph.parse(raw, ctx=ctx)
    t_parse = time.perf_counter() - t0
    n = net.n_nodes
    used = np.arange(n, dtype=np.uint32)
    lat = torch.empty(n * n, dtype=torch.int64, device="cuda")
    loss = torch.empty(n * n, dtype=torch.float32, device="cuda")

    def per_build(shortest):
        for _ in range(a.warmup):
            net.build_rows_device(used, 0, n, lat.data_ptr(), loss.data_ptr(), shortest)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            net.build_rows_device(used, 0, n, lat.data_ptr(), loss.data_ptr(), shortest)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / a.steps

    t_direct = per_build(False)
    t_build = per_build(True)  # the table left in lat/loss is the shortest-path one

    def one_shot():  # what a simulation pays for its one table: a fresh device graph (upload), plan, build
        fresh = NetworkGraph(n, net.edge_src, net.edge_dst, net.edge_latency_ns, net.edge_packet_loss, net.directed,
                             ctx=ctx)
        fresh.build_rows_device(used, 0, n, lat.data_ptr(), loss.data_ptr(), True)
        fresh.close()

    one_shot()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        one_shot()
    torch.cuda.synchronize()
    t_one_shot = (time.perf_counter() - t0) / a.steps
    # the arc sort runs once per graph (a rebuild reuses the sorted arcs): timed on a fresh graph
    ctx.enable_timers(True)
    queue_ahead(ctx, torch)
    one_shot()
    sort_ms, _, _ = ctx.read_timer("dense_sort")
    ctx.enable_timers(True)
    queue_ahead(ctx, torch)
    net.build_rows_device(used, 0, n, lat.data_ptr(), loss.data_ptr(), True)
    relax_ms, launches, _ = ctx.read_timer("relax")
    dense_ms, dense_n, _ = ctx.read_timer("sssp_dense")
    rec_b = ctx.read_timer("sssp_dense_rec_bytes")[2] / max(dense_n, 1)  # the library's arc record (12 B)
    ctx.enable_timers(True, count_work=True)  # (a separate build: the counting adds atomics)
    net.build_rows_device(used, 0, n, lat.data_ptr(), loss.data_ptr(), True)
    dense_rel = ctx.read_timer("sssp_dense")[2]
    ctx.enable_timers(False)
    n_arcs = int(2 * np.count_nonzero(g["src"] != g["dst"]))  # undirected: both directions
    roofline = None
    if dense_n:  # k_sssp_dense_lazy: one sorted-arc record (rec_b bytes, from the library) read (L2) per arc relaxed
        k_s = dense_ms / 1e3 / dense_n
        ach = rec_b * dense_rel / dense_n / k_s / 1e9
        pm = (pmc or {}).get("sssp_dense", {})
        roofline = {"kernel": "k_sssp_dense_lazy", "bound": "l2", "achieved": round(ach, 1), "peak": L2_PEAK_GBS,
                    "unit": "GB/s", "frac": round(ach / L2_PEAK_GBS, 4), "traffic": pm.get("hbm_bytes_per_launch"),
                    "avg_launch_ms": round(dense_ms / dense_n, 4), "arc_sort_ms": round(sort_ms, 4),
                    "relaxations_per_launch": dense_rel / dense_n, "record_bytes": rec_b,
                    "redundancy_vs_dijkstra": round(dense_rel / max(1.0, float(n) * n_arcs), 4),
                    "valu_frac_pmc": pm.get("valu_frac"),
                    "what": "relaxations = arcs read (the lazy search: each settled row resumed in whole "
                            "chunks up to the round's threshold); Dijkstra relaxes every arc of every "
                            "settled node (n x arcs)"}
    # value: a warm rebuild on the same device graph (the per-graph arc sort is cached in the
    # context); one_shot_s is the cold build a simulation pays once (sim_config.rs:137-141):
    # upload, arc sort, search
    leg = {"metric": "APSP routing build (s) @1.2k-node complete graph", "unit": "s", "value": round(t_build, 6),
           "value_kind": "warm rebuild (arcs sorted once per graph); one_shot_s is the cold build",
           "higher_is_better": False, "direct_paths_s": round(t_direct, 6), "gml_parse_s": round(t_parse, 4),
           "one_shot_s": round(t_one_shot, 6), "roofline": roofline,
           "relax_ms": round(relax_ms, 4), "relax_launches": launches,
           "config": {"workload": f"C2: {n}-node complete undirected graph from GML ({len(raw)} bytes), latency "
                                  "U[1,300] ms, self-loops U[1,10] ms, loss 0 w.p. 0.8 else U(0,0.02); every node "
                                  "used; use_shortest_path true", "nodes": n, "edges": int(len(g["src"]))}}
    if with_cpu:
        from oracle import oracle as O  # the checker, timed as the CPU baseline

        th = CPU_THREADS
        t0 = time.perf_counter()
        rc, olat, oloss, _ = O.shortest_paths(n, g["src"], g["dst"], g["lat"], g["loss"], False, used, threads=th)
        tc = time.perf_counter() - t0
        assert rc == 0
        leg["cpu_baseline"] = {"value": round(tc, 4), "unit": "s", "cores": th, "kind": "port", **CPU_INFO,
                               "sample": f"all {n} sources (binary-heap Dijkstra, dense output), {th} threads"}
        leg["speedup_vs_cpu"] = round(tc / t_build, 1)
        leg["parity_vs_cpu"] = bool(
            np.array_equal(lat.cpu().numpy().view(np.uint64).reshape(n, n), olat)
            and np.array_equal(loss.cpu().numpy().view(np.uint32).reshape(n, n), oloss.view(np.uint32)))
    return leg


def main():
    a = parse_args()
    D = Dist(a.gpus)
    torch = D.torch
    from shadow_amd import Context, NetworkGraph, synth
    from shadow_amd.worker import DeviceTable, HostTable, PacketBatch, Deliveries, deliver_round

    ctx = Context(D.local, stream=torch.cuda.current_stream().cuda_stream)
    # N > 1: the collectives go through the library (sg_comm_*: RCCL on the context's stream, the
    # calls INTEGRATION.md's Rust caller makes); SG_BENCH_COMM=torch keeps torch.distributed's
    comm = None
    if D.dist and os.environ.get("SG_BENCH_COMM", "sg") != "torch":
        from shadow_amd.comm import maybe_comm

        comm = maybe_comm(ctx, D.dist)
    collectives = ("sg_comm (RCCL through the C ABI)" if comm else
                   f"torch.distributed ({D.backend})" if D.dist else None)
    # the PMC summary was collected on the default workload: its per-launch bytes
    # describe no other configuration
    if a.config == "c5" and a.pmc_json == PMC_DEFAULT:
        a.pmc_json = PMC_C5
    pmc = load_pmc(a.pmc_json) if (a.config == "c3c4" and a.nodes == 10000) or a.config == "c5" else {}

    c5 = a.config == "c5"
    if c5:  # 10M packets per round in total, split over the ranks
        a.packets = (a.packets + D.world - 1) // D.world
    # ---------------- routing-table build (C3 / C5) ----------------
    g = synth.ring_chords_graph(a.nodes, a.degree, seed=1)
    net = NetworkGraph(g["n"], g["src"], g["dst"], g["lat"], g["loss"], g["directed"], ctx=ctx)
    used = np.arange(a.nodes, dtype=np.uint32)
    route_bal = None
    if D.world > 1:
        # the table's row order that gives every rank's row block an even share of the
        # sending hosts (synth.make_hosts puts host h on node h mod nodes): the same equal
        # row blocks, hosts partitioned by the rank holding their node's row
        from shadow_amd.dist import balanced_node_order

        order, route_bal = balanced_node_order(np.arange(a.hosts) % a.nodes, a.nodes, D.world)
        used = np.asarray(order, dtype=np.uint32)
    nu = len(used)
    rows = (nu + D.world - 1) // D.world
    r0, r1 = min(D.rank * rows, nu), min((D.rank + 1) * rows, nu)
    full_lat = torch.empty(D.world * rows * nu, dtype=torch.int64, device="cuda")
    full_loss = torch.empty(D.world * rows * nu, dtype=torch.float32, device="cuda")
    my_lat = full_lat[D.rank * rows * nu:(D.rank + 1) * rows * nu]
    my_loss = full_loss[D.rank * rows * nu:(D.rank + 1) * rows * nu]

    def build():
        # rows are independent units: each rank keeps its row shard (delivery reads only its own rows)
        net.build_rows_device(used, r0, r1, my_lat.data_ptr(), my_loss.data_ptr(), True)

    def build_fresh():
        # what a simulation pays for its one table (sim_config.rs:137-141): a new device graph
        # (sg_net_create: upload, CSC/CSR), the phase plan (on the device) and the search,
        # then the graph released (sg_net_destroy)
        fresh = NetworkGraph(g["n"], g["src"], g["dst"], g["lat"], g["loss"], g["directed"], ctx=ctx)
        fresh.build_rows_device(used, r0, r1, my_lat.data_ptr(), my_loss.data_ptr(), True)
        fresh.close()

    def allgather():
        if comm:  # in place: each rank's block is its own slice of full_lat / full_loss
            comm.allgather_rows(full_lat, full_loss, rows, nu)
            return
        if D.coll_dev == "cpu":  # gloo rehearsal: host-staged
            for full, mine in ((full_lat, my_lat), (full_loss, my_loss)):
                host = full.cpu()
                D.dist.all_gather_into_tensor(host, mine.cpu())
                full.copy_(host)
            return
        D.dist.all_gather_into_tensor(full_lat, my_lat)
        D.dist.all_gather_into_tensor(full_loss, my_loss)

    # the first build in the process also pays one-time HIP work (kernel loads, workspace)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    build_fresh()
    torch.cuda.synchronize()
    t_cold = time.perf_counter() - t0
    # the headline: one-shot builds in a warm process, each on a fresh graph with its own plan
    t_build = timed(D, build_fresh, a.steps, a.warmup)
    # beside it: rebuilds on the same device graph (the plan is rebuilt too; nothing is cached)
    t_warm = timed(D, build, a.steps, a.warmup)
    t_allgather = timed(D, allgather, max(1, a.steps // 2), 1) if D.dist else 0.0
    # The sharded build rehearsed on this one GPU: every rank's row block of an N-way split,
    # one-shot (upload, the block's own plan, search, release) as that rank would build it.
    # max_ms is the N-GPU build time less the all-gather; frac_of_linear = (one-shot / N) / max_ms.
    note(f"routing build timed: {t_build * 1e3:.3f} ms one-shot")
    rank_blocks = None
    if D.world == 1 and a.rank_blocks:
        rank_blocks = {}
        bl = torch.empty(((nu + 1) // 2) * nu, dtype=torch.int64, device="cuda")
        bf = torch.empty(((nu + 1) // 2) * nu, dtype=torch.float32, device="cuda")
        for N in (int(x) for x in a.rank_blocks.split(",") if x):
            per = (nu + N - 1) // N
            ts = []
            for r in range(N):
                b0, b1 = min(r * per, nu), min((r + 1) * per, nu)

                def one(b0=b0, b1=b1):
                    fresh = NetworkGraph(g["n"], g["src"], g["dst"], g["lat"], g["loss"], g["directed"], ctx=ctx)
                    fresh.build_rows_device(used, b0, b1, bl.data_ptr(), bf.data_ptr(), True)
                    fresh.close()
                ts.append(timed(D, one, 5, 2))
            rank_blocks[str(N)] = {"rows_per_rank": per, "max_ms": round(max(ts) * 1e3, 4),
                                   "per_rank_ms": [round(t * 1e3, 4) for t in ts],
                                   "linear_ms": round(t_build / N * 1e3, 4),
                                   "frac_of_linear": round(t_build / N / max(ts), 3)}
        del bl, bf
    # instrumented build on the kernel's own stream: HIP-event launch times, then
    # (separately, the counting variant is slower) the relaxations performed
    ctx.enable_timers(True)
    queue_ahead(ctx, torch)
    build()
    timers = {k: ctx.read_timer(k) for k in ("sssp", "sssp_bounded", "relax", "out", "relax_wide", "plan_sets",
                                             "plan_bounds", "sssp_bucket")}
    ctx.enable_timers(True, count_work=True)
    build()
    works = {k: ctx.read_timer(k)[2] for k in ("sssp", "relax", "sssp_bucket", "sssp_bucket_entries")}
    ctx.enable_timers(False)
    n_arcs = int(net.edge_src.size * 2 - 2 * np.count_nonzero(net.edge_src == net.edge_dst))
    rows_mine = r1 - r0
    dijkstra_relax = float(rows_mine) * n_arcs  # per-source Dijkstra: every arc of every source once
    lds = timers["sssp"][1] > 0
    band = timers["sssp_bucket"][1] > 0
    pm = pmc.get("sssp" if lds else "sssp_band" if band else "relax", {})
    if band:
        # k_sssp_band (sg_bucket.hip, graphs past the LDS search): per relaxation a 12-B arc record
        # (L2 / Infinity Cache); per arena entry 12 B written and 12 B read; per cell the settled key
        # written to and read from the scratch row (8 + 8 B) and the 12-B table cell written
        k_ms, k_n, _ = timers["sssp_bucket"]
        k_s = k_ms / 1e3 / max(k_n, 1)
        relax_per_launch = works["sssp_bucket"] / max(k_n, 1)
        entries = works["sssp_bucket_entries"] / max(k_n, 1)
        cells = float(rows_mine) * nu / max(k_n, 1)
        alg = ARC_BYTES_PER_RELAX * relax_per_launch + 24.0 * entries + 28.0 * cells
        achieved = alg / k_s / 1e9 if k_n else 0.0
        # PMC of the largest dispatch: bench's rank-block leg launches the kernel on 1/8 of the rows
        # too, so the per-dispatch average mixes sizes; the one-shot build is the largest dispatch
        big = pm.get("largest", {})
        roofline = {"kernel": "k_sssp_band", "bound": "l2", "achieved": round(achieved, 1), "peak": L2_PEAK_GBS,
                    "unit": "GB/s", "frac": round(achieved / L2_PEAK_GBS, 4),
                    "traffic": big.get("hbm_bytes", pm.get("hbm_bytes_per_launch")),
                    "traffic_write_bytes": big["write_kb"] * 1024 if "write_kb" in big else None,
                    "traffic_fetch_bytes_raw": big["fetch_kb_raw"] * 1024 if "fetch_kb_raw" in big else None,
                    "algorithmic_bytes_per_launch": alg, "avg_launch_ms": round(k_s * 1e3, 4),
                    "launches_per_build": k_n, "relaxations_per_launch": relax_per_launch,
                    "arena_entries_per_launch": entries,
                    "redundancy_vs_dijkstra": round(relax_per_launch * max(k_n, 1) / max(dijkstra_relax, 1.0), 3),
                    "valu_frac_pmc": big.get("valu_frac", pm.get("valu_frac")),
                    "hbm_view": {"achieved": round(alg / k_s / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                 "frac": round(alg / k_s / 1e9 / HBM_PEAK_GBS, 4),
                                 "what": "the same algorithmic bytes against HBM (arena and table pass HBM; "
                                         "the arcs sit in L2 / the Infinity Cache)"}}
    elif lds:
        # k_sssp_lds: a 12-B arc record gathered from L2 per relaxation; its HBM
        # traffic is the 12-B (latency, loss) cell per table entry.  A build is one
        # launch, or three (the bounded phases, timer sssp_bounded): per-launch
        # figures average over all of them, as rocprof's kernel average does
        k_ms = timers["sssp"][0] + timers["sssp_bounded"][0]
        k_n = timers["sssp"][1] + timers["sssp_bounded"][1]
        k_s = k_ms / 1e3 / max(k_n, 1)
        relax_per_launch = works["sssp"] / max(k_n, 1)
        gather_bytes = ARC_BYTES_PER_RELAX * relax_per_launch
        out_bytes = 12.0 * rows_mine * nu / max(k_n, 1)
        achieved = gather_bytes / k_s / 1e9 if k_n else 0.0
        roofline = {"kernel": "k_sssp_lds", "bound": "l2", "achieved": round(achieved, 1), "peak": L2_PEAK_GBS,
                    "unit": "GB/s", "frac": round(achieved / L2_PEAK_GBS, 4), "traffic": pm.get("hbm_bytes_per_launch"),
                    "algorithmic_bytes_per_launch": gather_bytes + out_bytes,
                    "avg_launch_ms": round(k_s * 1e3, 4), "launches_per_build": k_n,
                    "phase_ms": {"unbounded": round(timers["sssp"][0], 4),
                                 "bounded": round(timers["sssp_bounded"][0], 4)},
                    "relaxations_per_launch": relax_per_launch,
                    "redundancy_vs_dijkstra": round(relax_per_launch * max(k_n, 1) / max(dijkstra_relax, 1.0), 3),
                    "valu_frac_pmc": pm.get("valu_frac"),
                    "hbm_view": {"achieved": round(out_bytes / k_s / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                 "frac": round(out_bytes / k_s / 1e9 / HBM_PEAK_GBS, 4),
                                 "what": "the row-major table written (12 B per cell)"}}
    else:
        relax_ms, relax_launches, _ = timers["relax"]
        avg_launch_s = relax_ms / 1e3 / max(relax_launches, 1)
        relax_per_launch = works["relax"] / max(relax_launches, 1)
        # the 512-B key rows every relaxed in-arc gathers from the batch slab (L2 / Infinity Cache)
        gather_bytes = ROW_BYTES_PER_RELAX * relax_per_launch
        achieved = gather_bytes / avg_launch_s / 1e9 if relax_launches else 0.0
        roofline = {"kernel": "k_relax_w2", "bound": "l2", "achieved": round(achieved, 1), "peak": L2_PEAK_GBS,
                    "unit": "GB/s", "frac": round(achieved / L2_PEAK_GBS, 4), "traffic": pm.get("hbm_bytes_per_launch"),
                    "algorithmic_bytes_per_launch": gather_bytes,
                    "avg_launch_ms": round(avg_launch_s * 1e3, 4), "launches_per_build": relax_launches,
                    "lane_relaxations_per_launch": relax_per_launch,
                    "redundancy_vs_dijkstra": round(relax_per_launch * relax_launches / max(dijkstra_relax, 1.0), 3),
                    "valu_frac_pmc": pm.get("valu_frac")}
        if pm.get("hbm_bytes_per_launch") and relax_launches:
            hbm = pm["hbm_bytes_per_launch"] / avg_launch_s / 1e9
            roofline["hbm_view"] = {"achieved": round(hbm, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                    "frac": round(hbm / HBM_PEAK_GBS, 4)}
    # the batched-source slab kernel on the same rows, for comparison (the default above 10.9k nodes)
    t_slab = None
    t_unbounded = None
    if (lds or band) and not a.no_compare:
        os.environ["SG_APSP_LDS"] = "0"
        t_slab = timed(D, build, max(1, a.steps // 2), 1)
        os.environ.pop("SG_APSP_LDS")
        if lds:  # and the LDS search in one launch with every key from infinity (no bound rows)
            os.environ["SG_SSSP_SEEDS"] = "0"
            t_unbounded = timed(D, build, max(1, a.steps // 2), 1)
            os.environ.pop("SG_SSSP_SEEDS")

    # end to end: the whole table into the dense host RoutingInfo (sg_routing_info_fill:
    # row blocks built on the GPU, copied into pinned host memory while the next builds)
    note("instrumented builds and comparisons done")
    e2e = None
    if D.world == 1 and not a.no_e2e:
        from shadow_amd import RoutingInfo

        ri = RoutingInfo(np.arange(nu, dtype=np.uint32))
        ri.fill(net, used, True)  # warm-up (and the pinned pages touched once)
        torch.cuda.synchronize()
        reps = max(1, a.steps // 2)
        t0 = time.perf_counter()
        for _ in range(reps):
            ri.fill(net, used, True)
        t_e2e = (time.perf_counter() - t0) / reps
        same = bool(np.array_equal(ri.latency_ns[: r1 - r0], my_lat.cpu().numpy().view(np.uint64).reshape(-1, nu)[
                    : r1 - r0]))
        # the host table holds 8-byte cells (latency << 32 | bits(loss); sg_route_info.hip)
        e2e = {"ms": round(t_e2e * 1e3, 3), "pinned": ri.pinned, "table_bytes": 8 * nu * nu,
               "d2h_GBs": round(8.0 * nu * nu / t_e2e / 1e9, 1), "same_as_device_table": same,
               "what": "sg_routing_info_fill: kernel + D2H of the whole table into the dense host RoutingInfo"}
        del ri

    note("end-to-end RoutingInfo fill done")
    cpu = None
    parity = None
    cpu_faithful = None
    if D.rank == 0 and D.world == 1 and not a.no_cpu:
        from oracle import oracle as O  # the checker, timed as the CPU baseline

        threads = CPU_THREADS
        k = nu if a.cpu_rows <= 0 else min(a.cpu_rows, nu)
        t0 = time.perf_counter()
        rc, olat, oloss, _ = O.shortest_paths(g["n"], g["src"], g["dst"], g["lat"], g["loss"], False, used,
                                              rows=(0, k), threads=threads)
        t_cpu = (time.perf_counter() - t0) * nu / k
        assert rc == 0
        # parity at the headline size: the GPU's rows [0, k) against the CPU's, every cell
        glat = my_lat.cpu().numpy().view(np.uint64).reshape(-1, nu)[:k]
        gloss = my_loss.cpu().numpy().view(np.uint32).reshape(-1, nu)[:k]
        parity = bool(np.array_equal(glat, olat) and np.array_equal(gloss, oloss.view(np.uint32)))
        del olat, oloss, glat, gloss
        what = f"all {nu} sources" if k == nu else f"the first {k} of {nu} sources, scaled by {nu}/{k}"
        cpu = {"value": round(t_cpu, 4), "unit": "s", "cores": threads, "kind": "port", **CPU_INFO,
               "sample": f"{what} (binary-heap Dijkstra, dense output, no HashMap materialisation) "
                         f"on the same graph, {threads} threads"}
        # the reference's own cost: SipHash score maps, nodes.contains filter, per-source and
        # global HashMaps, self pairs, the id remap (oracle/sg_faithful.c), on a bounded sample
        kf = min(nu, C5_FAITHFUL_ROWS if c5 else FAITHFUL_ROWS)
        rcf, _, _, ph = O.routing_faithful(g["n"], g["src"], g["dst"], g["lat"], g["loss"], False, used, rows=kf,
                                           threads=threads, read_back=False)
        assert rcf == 0
        t_f = sum(ph) * nu / kf
        cpu_faithful = {"value": round(t_f, 3), "unit": "s", "cores": threads, "kind": "port", **CPU_INFO,
                        "phases_s": {"dijkstra_filter_per_source_maps": round(ph[0] * nu / kf, 3),
                                     "global_collect": round(ph[1] * nu / kf, 3),
                                     "self_pairs": round(ph[2] * nu / kf, 4),
                                     "id_remap_map": round(ph[3] * nu / kf, 3)},
                        "sample": f"the first {kf} of {nu} sources through the reference's own steps "
                                  "(graph/mod.rs:183-228, sim_config.rs:411-448), each phase scaled by "
                                  f"{nu}/{kf}, {threads} threads"}
        # the same two baselines on every logical core the host shows (rayon's default pool);
        # on a GPU box that is more threads than this job's CPU share, so they oversubscribe it
        tv = CPU_INFO["nproc_visible"]
        if tv != threads:
            t0 = time.perf_counter()
            rc, _, _, _ = O.shortest_paths(g["n"], g["src"], g["dst"], g["lat"], g["loss"], False, used,
                                           rows=(0, k), threads=tv)
            t_all = (time.perf_counter() - t0) * nu / k
            rcf, _, _, ph = O.routing_faithful(g["n"], g["src"], g["dst"], g["lat"], g["loss"], False, used, rows=kf,
                                               threads=tv, read_back=False)
            cpu_all = {"threads": tv, "share": threads, "dense_port_s": round(t_all, 4),
                       "faithful_s": round(sum(ph) * nu / kf, 3),
                       "what": "the dense port and the faithful variant on all logical cores, same samples; "
                               f"the job's CPU share is {threads}, so these oversubscribe it"}
        else:
            cpu_all = {"threads": tv, "share": threads, "what": "all logical cores are the share: the runs above"}
        cpu_faithful["all_cores"] = cpu_all

    result = {
        "metric": METRIC, "value": round(t_build, 6), "unit": "s", "n_gpus": D.world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(t_build * 1e3, 4), "higher_is_better": False,
        "scaling": "strong", "vs_baseline": None, "dtype": "u64+f32",
        "data": f"synthetic (seeded ring+chords graph, SURVEY §8d {'C5' if c5 else 'C3'})",
        "config": {"workload": f"{'C5' if c5 else 'C3'} APSP routing build: {a.nodes // 1000}k-node undirected "
                               "ring+chords graph, mean degree 8, "
                               "latency U[1,100] ms (integer us), loss 0 w.p. 0.8 else U(0,0.02); all nodes used; "
                               "source rows sharded across ranks (each rank keeps its row block; the optional RCCL "
                               "all-gather of the blocks is timed separately in apsp_detail.allgather_ms)",
                   "nodes": a.nodes, "arcs": n_arcs, "parallelism": f"rows{D.world}"},
        "roofline": roofline, "cpu_baseline": cpu,
        "parity_vs_cpu": parity,
        "apsp_detail": {"kernel": roofline["kernel"],
                        "slab_kernel_ms": round(t_slab * 1e3, 4) if t_slab else None,
                        "unbounded_one_launch_ms": round(t_unbounded * 1e3, 4) if t_unbounded else None,
                        "value_is": "one-shot build: sg_net_create + plan + search + sg_net_destroy per step",
                        "same_graph_rebuild_ms": round(t_warm * 1e3, 4),
                        "plan_ms": round(timers["plan_sets"][0] + timers["plan_bounds"][0], 4),
                        "plan_kernels_ms": {"plan_sets": round(timers["plan_sets"][0], 4),
                                            "plan_bounds": round(timers["plan_bounds"][0], 4)},
                        "cold_build_ms": round(t_cold * 1e3, 4),
                        "out_kernel_ms": round(timers["out"][0], 4),
                        "wide_rows_ms": round(timers["relax_wide"][0], 4),
                        "allgather_ms": round(t_allgather * 1e3, 4),
                        "rank_block_ms": rank_blocks,
                        "table_bytes": 12 * nu * nu,
                        "end_to_end": e2e,
                        "cpu_baseline_faithful": cpu_faithful},
    }
    if cpu:
        result["apsp_detail"]["speedup_vs_cpu"] = round(cpu["value"] / t_build, 1)
    if cpu_faithful:
        result["apsp_detail"]["speedup_vs_cpu_faithful"] = round(cpu_faithful["value"] / t_build, 1)
        if e2e:
            result["apsp_detail"]["speedup_vs_cpu_faithful_end_to_end"] = round(cpu_faithful["value"] / (e2e["ms"] / 1e3), 1)
    if D.rank == 0 and not a.no_gml:
        note("GML ingest leg")
        result["gml_ingest"] = gml_leg(a, NetworkGraph, synth)
    if D.rank == 0 and not a.no_c2:
        note("C2 leg")
        result["c2"] = c2_leg(a, ctx, torch, NetworkGraph, synth, D.world == 1 and not a.no_cpu, pmc)

    note("delivery leg")
    # ---------------- delivery round (C4) ----------------
    if not a.no_delivery:
        from shadow_amd.dist import HostPartition, ShardedDelivery

        hosts = synth.make_hosts(a.hosts, a.nodes, general_seed=1, exact_seeds=True)
        if route_bal is not None:  # host -> its node's row in the balanced order
            hosts["route"] = np.asarray(route_bal, dtype=np.uint32)
        part = HostPartition(hosts["route"], nu, D.world)
        mine = part.hosts_of[D.rank]
        # weak scaling: each rank sends a.packets from the hosts it owns, to destinations anywhere
        pk = synth.make_packets(a.packets, hosts, T0 + 10**9, T0 + 10**9 + 10**6, seed=100 + D.rank,
                                src_hosts=mine)
        ht = HostTable(hosts["ip"], hosts["route"], hosts["seed"], ctx=ctx)
        table = DeviceTable(my_lat, my_loss, nu, r0)
        t_pack = None
        if not a.no_pack:  # once per routing table, outside the per-round timing (sg_table_pack)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            packed = table.pack(ctx)
            torch.cuda.synchronize()
            t_pack = time.perf_counter() - t0 if packed else None
        batch = PacketBatch.from_numpy(pk["src"], pk["dst_ip"], pk["payload"], pk["send_time"])
        src_global = pk["src"]
        out = Deliveries.allocate(a.packets, a.hosts)
        round_end, sim_end = T0 + 10**9 + 10**6, 2**63
        # padded: after the first (warm-up) round, the fixed-split exchange with one host sync per round
        sharded = ShardedDelivery(ctx, ht, table, part, D.rank, D.world, dist=comm or D.dist,
                                  padded=not a.exact_exchange) if D.world > 1 else None

        def rnd():
            if sharded:
                sharded.round(batch, round_end, sim_end, 0)
            else:
                deliver_round(ht, table, batch, round_end, sim_end, 0, out=out, ctx=ctx)

        # a round is ~0.1 ms: at least 100 of them, so one host-side hiccup moves the mean little
        t_round = timed(D, rnd, max(a.steps, SUB_MS_REPS), a.warmup)
        note(f"delivery round timed: {t_round * 1e3:.4f} ms")
        per_rank = None
        if sharded:  # load balance of the host partition: packets sent, records sent / received per rank
            mine_c = [float(a.packets), float(sum(sharded.last_send_counts)), float(sum(sharded.last_recv_counts))]
            allc = D.gather(mine_c)
            per_rank = {"packets": [int(x[0]) for x in allc], "records_sent": [int(x[1]) for x in allc],
                        "records_received": [int(x[2]) for x in allc], "exchange": sharded.last_mode,
                        "padded_cap": sharded.cap}
        t_pcie = None
        if D.world == 1:
            # the boundary takes device buffers; a caller holding the packet log in host memory
            # also pays H2D of the inputs (20 B/packet) and D2H of the outputs (status, time, id,
            # order, offsets): timed here from pinned host buffers, never the headline value
            h_in = [t.cpu().pin_memory() for t in (batch.src_host, batch.dst_ipv4, batch.payload_len,
                                                   batch.send_time_ns)]
            h_out = [t.cpu().pin_memory() for t in (out.status, out.deliver_time_ns, out.event_id, out.dst_order,
                                                    out.dst_offsets)]

            def rnd_pcie():
                for d, hsrc in zip((batch.src_host, batch.dst_ipv4, batch.payload_len, batch.send_time_ns), h_in):
                    d.copy_(hsrc, non_blocking=True)
                deliver_round(ht, table, batch, round_end, sim_end, 0, out=out, ctx=ctx)
                for hdst, d in zip(h_out, (out.status, out.deliver_time_ns, out.event_id, out.dst_order,
                                           out.dst_offsets)):
                    hdst.copy_(d, non_blocking=True)

            t_pcie = timed(D, rnd_pcie, max(3, a.steps // 4), 1)
        ctx.enable_timers(True)
        queue_ahead(ctx, torch)
        rnd()
        kt = {k: ctx.read_timer(k) for k in ("seg_bounds", "walk", "scan", "scatter", "scatter2", "sort_small",
                                             "sort_big", "pack", "rec_count", "rec_scatter")}
        ctx.enable_timers(False)
        walk_ms, walk_n, walk_bytes = kt["walk"]
        walk_s = walk_ms / 1e3 / max(walk_n, 1)
        ach = walk_bytes / max(walk_n, 1) / walk_s / 1e9 if walk_n else 0.0
        total_pkts = D.sum(float(a.packets))
        # SURVEY §8d algorithmic bytes per round (the packed path key gathers 8 B instead of 12 B)
        round_bytes = (41.0 if table.path_key is not None else 45.0) * a.packets + 84.0 * a.hosts
        pmw = pmc.get("walk", {})
        delivery = {
            "metric": "packets routed/sec per sim round", "value": round(total_pkts / t_round, 1),
            "unit": "packets/s", "higher_is_better": True, "ms_per_round": round(t_round * 1e3, 4),
            "scaling": "strong" if c5 else "weak", "dtype": "u64+f32+f64",
            "config": {"workload": f"{'C5' if c5 else 'C4'} delivery round: {a.hosts // 1000}k hosts on the "
                                   f"{a.nodes // 1000}k-node graph (node h mod {a.nodes // 1000}k), {a.packets} "
                                   "packets per rank from the hosts it owns, dst uniform over all hosts != src, "
                                   "20% zero-payload, "
                                   "send_time U[1 ms round)" + (
                                       ("; records exchanged by RCCL all-to-all to the destination's owner"
                                        if D.coll_dev == "cuda" else "; records exchanged by a host-staged gloo "
                                        "all-to-all (a rehearsal: not a measurement)") if D.world > 1 else ""),
                       "hosts": a.hosts, "packets_per_rank": a.packets},
            "roofline": {"kernel": "k_walk", "bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": pmw.get("hbm_bytes_per_launch"),
                         "avg_launch_ms": round(walk_s * 1e3, 4), "valu_frac_pmc": pmw.get("valu_frac"),
                         "rocprof": rocprof_view(pmw, walk_bytes / max(walk_n, 1))},
            "round_hbm_GBs": round(round_bytes / t_round / 1e9, 1),
            "per_rank": per_rank,
            "parallelism": f"hosts{D.world}",
            "path_key_table": table.path_key is not None,
            "pcie_inclusive_ms_per_round": round(t_pcie * 1e3, 4) if t_pcie is not None else None,
            "table_pack_ms": round(t_pack * 1e3, 4) if t_pack is not None else None,
            "kernel_ms": {k: round(v[0] / max(v[1], 1), 4) for k, v in kt.items()},
        }
        if D.rank == 0 and D.world == 1 and not a.no_cpu:
            from oracle import oracle as O

            lat_h = my_lat.cpu().numpy().view(np.uint64).reshape(-1, nu)[: r1 - r0]
            loss_h = my_loss.cpu().numpy().reshape(-1, nu)[: r1 - r0]
            rng0 = np.stack([O.xoshiro_seed(int(s)) for s in hosts["seed"]]).astype(np.uint64)
            ctr0 = np.zeros(a.hosts, np.uint64)
            th = CPU_THREADS  # the box's CPU share (16 logical CPUs per GPU)
            note("delivery: CPU baseline round")
            orng, octr = rng0.copy(), ctr0.copy()
            t0 = time.perf_counter()
            wr = O.deliver_round(round_end, sim_end, 0, src_global, pk["dst_ip"], pk["payload"], pk["send_time"],
                                 hosts["ip"], hosts["route"], lat_h, loss_h, orng, octr, threads=th)
            tc = time.perf_counter() - t0
            # parity at the benchmarked size: the same round from the seed state on the GPU,
            # every per-packet output, the buckets, the minima and the hosts' RNG / counters
            ht.set_state(rng0, ctr0)
            st = deliver_round(ht, table, batch, round_end, sim_end, 0, out=out, ctx=ctx)
            got = out.to_numpy(a.packets)
            grng, gctr = ht.get_state()
            same = all(np.array_equal(got[k], wr[k]) for k in ("status", "deliver_time", "event_id", "dst_order",
                                                                "dst_offsets"))
            same = same and got["delivered"] == wr["delivered"] and got["min_deliver"] == wr["min_deliver"]
            same = same and got["min_lat"] == wr["min_lat"]
            same = same and np.array_equal(grng, orng) and np.array_equal(gctr, octr)
            delivery["parity_vs_cpu"] = bool(same)
            del st
            delivery["cpu_baseline"] = {"value": round(a.packets / tc, 1), "unit": "packets/s", "cores": th,
                                        "kind": "port", **CPU_INFO, "sample": f"one full round of {a.packets} packets, "
                                        "send_packet semantics + per-destination EventQueue order; source hosts "
                                        f"split over {th} threads as Shadow's workers split hosts"}
            delivery["speedup_vs_cpu"] = round(delivery["value"] / delivery["cpu_baseline"]["value"], 1)
            # the reference's own per-packet costs on the same round (oracle/sg_faithful.c): SipHash
            # Dns / IpAssignment / RoutingInfo lookups (a map of every node pair), the global
            # RwLock'd packet counter, a mutex'd binary heap per destination queue
            frng, fctr = rng0.copy(), ctr0.copy()
            note("delivery: faithful CPU baseline round" + (" skipped at C5" if c5 else ""))
        if D.rank == 0 and D.world == 1 and not a.no_cpu and not c5:
            # (C5: the reference's node-pair map would hold 2.5e9 entries; the dense port above is
            # the C5 baseline)
            fr = O.deliver_faithful(round_end, sim_end, 0, src_global, pk["dst_ip"], pk["payload"], pk["send_time"],
                                    hosts["ip"], hosts["route"], lat_h, loss_h, frng, fctr, threads=th)
            fsame = all(np.array_equal(fr[k], wr[k]) for k in ("status", "deliver_time", "event_id", "dst_order",
                                                               "dst_offsets"))
            fsame = fsame and np.array_equal(frng, orng) and np.array_equal(fctr, octr)
            delivery["cpu_baseline_faithful"] = {
                "value": round(a.packets / fr["round_s"], 1), "unit": "packets/s", "cores": th, "kind": "port",
                **CPU_INFO, "setup_s": round(fr["setup_s"], 2), "matches_dense_cpu": bool(fsame),
                "sample": f"the same round of {a.packets} packets through Worker::send_packet on the reference's "
                          "structures (worker.rs:322-397, :517-607; graph/mod.rs:354-456; dns.rs:176): "
                          f"{nu}x{nu} node-pair SipHash map, hosts round-robin over {th} threads; setup_s = "
                          "building the maps (startup in the reference), not in the value"}
            delivery["speedup_vs_cpu_faithful"] = round(delivery["value"] / delivery["cpu_baseline_faithful"]["value"],
                                                        1)
            del fr
        result["delivery"] = delivery
        if not a.no_codel:
            buckets = round_buckets(out, pk["payload"], sharded)
            note("CoDel leg")
            result["codel"] = codel_leg(a, D, ctx, torch, buckets, a.packets, pmc)
            note("inbound leg")
            result["inbound"] = inbound_leg(a, D, ctx, torch, buckets, a.packets, pmc, round_end)
            note("outbound leg")
            result["outbound"] = outbound_leg(a, D, ctx, torch, pk, hosts, ht, table, round_end, sharded, pmc)

    result["collectives"] = collectives
    if D.rank == 0:
        print(json.dumps(result), flush=True)
    if comm:
        comm.close()
    if D.dist:
        D.dist.destroy_process_group()


if __name__ == "__main__":
    main()
