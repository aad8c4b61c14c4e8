"""Host HIP API calls and kernels of one window of a rocprofv3 --hip-trace --kernel-trace run, on one
clock: what the host does between a build's launches.
usage: python tools/host_api_timeline.py TRACE_DIR FIRST_KERNEL_SUBSTRING [NTH_FROM_END]
   prints, from the NTH_FROM_END-last dispatch of FIRST_KERNEL_SUBSTRING (default 2) to the next
   one, every API call (start, duration) and kernel (start, duration) in time order."""
import csv
import glob
import os
import sys


def main():
    d, first = sys.argv[1], sys.argv[2]
    nth = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    ev = []
    for f in glob.glob(os.path.join(d, "**", "*hip_api_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "api", r["Function"]))
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "gpu", r["Kernel_Name"].split("(")[0]))
    ev.sort()
    starts = [e[0] for e in ev if e[2] == "gpu" and first in e[3]]
    t0 = starts[-nth]
    t1 = starts[-nth + 1] if nth > 1 else ev[-1][1]
    # from the API call that launched it: the last launch call before the kernel start
    api_before = [e for e in ev if e[2] == "api" and e[0] <= t0 and "Launch" in e[3]]
    ta = api_before[-1][0] if api_before else t0
    for s, e, kind, name in ev:
        if ta <= s < t1:
            print(f"{(s - ta) / 1e3:10.2f} us  {kind}  {(e - s) / 1e3:9.2f} us  {name[-60:]}")


if __name__ == "__main__":
    main()
