#!/usr/bin/env python3
"""Why bench.py's HIP-event time of k_inbound differed from rocprof's (VERDICT r05 Weak #6):
the C4-sized inbound window (100k hosts, ~1M arrivals, 1 Gbit/s relays) through fresh
pipelines, the library's event timer read per call, in both call forms, with and without a
spin kernel queued ahead, next to the same calls' kernel-trace durations (run this under
rocprofv3 --kernel-trace and read the trace with tools/lane_trace.py)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from shadow_amd import Context
    from shadow_amd.router import InboundPipeline

    ctx = Context(0, stream=torch.cuda.current_stream().cuda_stream)
    rng = np.random.default_rng(1)
    H, N = 100_000, 990_000
    T0 = 946684800 * 10**9 + 10**9
    host = np.sort(rng.integers(0, H, N)).astype(np.uint32)
    t = (T0 + 10**6 + rng.integers(0, 300 * 10**6, N)).astype(np.uint64)
    o = np.lexsort((t, host))
    host, t = host[o], t[o]
    pkt = rng.permutation(N).astype(np.uint32)
    ln = rng.choice(np.array([28, 1476], np.uint32), N)
    dev = lambda x, dt, tv: torch.from_numpy(np.ascontiguousarray(x, dtype=dt).view(tv)).cuda()
    args = (dev(host, np.uint32, np.int32), dev(t, np.uint64, np.int64), dev(pkt, np.uint32, np.int32),
            dev(ln, np.uint32, np.int32))
    wend = int(t.max()) + 1
    bw = np.full(H, 10**9, np.uint64)
    fwd = torch.full((N,), -1, dtype=torch.int64, device="cuda")
    st = torch.zeros(N, dtype=torch.uint8, device="cuda")
    a_fwd = torch.full((N,), -1, dtype=torch.int64, device="cuda")
    a_st = torch.zeros(N, dtype=torch.uint8, device="cuda")
    pipes = [InboundPipeline(bw, 256, ctx=ctx) for _ in range(24)]
    it = iter(pipes)

    def call(ordered):
        p = next(it)
        if ordered:
            p.run_ordered(*args, wend, 0, 2**63, fwd, st, a_fwd, a_st)
        else:
            p.run(*args, wend, 0, 2**63, fwd, st)

    for ordered in (True, False):
        call(ordered)  # warm
    for ahead in (True, False):
        for ordered in (True, False):
            ts = []
            for _ in range(4):
                ctx.enable_timers(True)
                if ahead:
                    s = torch.cuda.ExternalStream(ctx.stream) if ctx.stream else torch.cuda.current_stream()
                    with torch.cuda.stream(s):
                        torch.cuda._sleep(2_000_000)
                call(ordered)
                ts.append(ctx.read_timer("inbound")[0] * 1e3)
                ctx.enable_timers(False)
            print(f"queue_ahead={ahead} ordered={ordered}: event us per call {[round(x, 1) for x in ts]}", flush=True)


if __name__ == "__main__":
    main()
