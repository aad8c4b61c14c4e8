#!/usr/bin/env python3
"""Print the kernels of a rocprofv3 --kernel-trace CSV in start order: name, duration and the
idle time since the previous kernel ended (us).  usage: trace_seq.py DIR [substring ...]"""
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
keep = sys.argv[2:]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
prev = None
for r in rows:
    n = r["Kernel_Name"]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if not keep or any(k in n for k in keep):
        print(f"{n.split('(')[0][-48:]:48s} {(e - s) / 1e3:9.1f} us  idle before {((s - prev) / 1e3) if prev else 0:9.1f} us")
    prev = e
