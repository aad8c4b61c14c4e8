"""Mean duration per (kernel, grid size) from a rocprofv3 --kernel-trace CSV: tells the launches of
one kernel apart when they differ by grid (e.g. the dense search's seed and seeded launches).
usage: python tools/kernel_grid_stats.py TRACE_DIR_OR_CSV [NAME_SUBSTRING]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    files = [path] if path.endswith(".csv") else glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)
    acc = defaultdict(list)
    for f in files:
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", "")
            if sub not in name:
                continue
            grid = r.get("Grid_Size_X") or r.get("Grid_Size") or "?"
            wg = r.get("Workgroup_Size_X") or r.get("Workgroup_Size") or "1"
            try:
                blocks = int(grid) // max(1, int(wg))
            except ValueError:
                blocks = grid
            acc[(name.split("(")[0], blocks)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for (name, blocks), d in sorted(acc.items(), key=lambda x: (x[0][0], str(x[0][1]))):
        d.sort()
        print(f"{name:40s} blocks {blocks!s:>8s} n {len(d):5d} mean {sum(d) / len(d):9.2f} us  "
              f"median {d[len(d) // 2]:9.2f} us")


if __name__ == "__main__":
    main()
