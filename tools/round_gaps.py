#!/usr/bin/env python3
"""Where a delivery round's wall time goes between its kernels: reads a rocprofv3
--kernel-trace CSV of tools/round_c4.py (20 timed rounds) and prints, per round, the kernels'
busy time, the gaps between consecutive kernels of the round, and the idle time before the
round's first kernel (the host's synchronisation return + the next round's first dispatch).
usage: python tools/round_gaps.py DIR (a rocprofv3 -d directory)"""
import csv
import glob
import sys

import numpy as np

ROUND_FIRST = ("k_host_off4", "k_host_off")


def main():
    f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
    rounds, cur = [], []
    for k in ks:
        name = k[2].split("(")[0].split("<")[0].replace("sg::", "").replace("void ", "").strip()
        if name in ROUND_FIRST and cur:
            rounds.append(cur)
            cur = []
        cur.append((k[0], k[1], name))
    rounds.append(cur)
    rounds = [r for r in rounds if r[0][2] in ROUND_FIRST][-20:]
    busy, inner, lead, names = [], [], [], None
    for i, r in enumerate(rounds):
        busy.append(sum(e - s for s, e, _ in r) / 1e3)
        inner.append(sum(max(0, r[j + 1][0] - r[j][1]) for j in range(len(r) - 1)) / 1e3)
        if i:
            lead.append((r[0][0] - rounds[i - 1][-1][1]) / 1e3)
        names = [n for _, _, n in r]
    gaps = np.array([[(r[j + 1][0] - r[j][1]) / 1e3 for j in range(len(r) - 1)] for r in rounds if len(r) == len(names)])
    print("kernels per round:", " -> ".join(names))
    print(f"busy {np.median(busy):.2f} us, gaps inside the round {np.median(inner):.2f} us "
          f"(per gap {np.round(np.median(gaps, axis=0), 2).tolist()}), idle before the round's first kernel "
          f"{np.median(lead):.2f} us; round period {np.median(busy) + np.median(inner) + np.median(lead):.2f} us")


if __name__ == "__main__":
    main()
