#!/usr/bin/env python3
"""Random-gather floor of the C5 path-cell read: G random 8-B reads from an
n x n u64 table (50k x 50k = 20 GB) with torch's index kernel, one read per
packet -- what k_walk's path gather can at best approach at C5.  Also times the
same count of reads from a 0.8 GB table (C4's 10k x 10k) for comparison.
python tools/gather_floor.py [--gathers 10000000]"""
import argparse
import time

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gathers", type=int, default=10_000_000)
    a = ap.parse_args()
    for n in (50000, 10000):
        tab = torch.empty(n * n, dtype=torch.int64, device="cuda")
        tab.fill_(7)
        idx = torch.randint(0, n * n, (a.gathers,), device="cuda", dtype=torch.int64)
        out = torch.empty(a.gathers, dtype=torch.int64, device="cuda")
        for _ in range(3):
            torch.index_select(tab, 0, idx, out=out)
        torch.cuda.synchronize()
        ts = []
        for _ in range(10):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            torch.index_select(tab, 0, idx, out=out)
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        ms = sorted(ts)[len(ts) // 2]
        print(f"table {n}x{n} ({n * n * 8 / 1e9:.1f} GB): {a.gathers} random 8-B gathers in {ms:.4f} ms "
              f"= {a.gathers / ms / 1e6:.2f} G gathers/s", flush=True)
        del tab, idx, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
