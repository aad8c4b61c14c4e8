#!/bin/bash
# Kernel-trace stats of the lane-per-host kernels (k_codel, k_inbound, k_outbound,
# k_out_compact, k_walk) from a short bench run without the CPU legs.
# usage (GPU box): bash tools/lane_stats.sh TAG
set -u
TAG=${1:-x}
export TMPDIR=/tmp
OUT=gpurun_out/lane_$TAG
mkdir -p $OUT
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 bench.py --no-cpu --no-gml --no-c2 --steps 5 --warmup 2 > $OUT/bench.log 2>&1 || { echo "stats run failed"; tail -5 $OUT/bench.log; exit 1; }
python3 - $OUT <<'PY'
import csv, glob, re, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"]
    if any(k in n for k in ("k_codel", "k_inbound", "k_outbound", "k_out_compact", "k_walk")):
        k = re.search(r"k_\w+(<[^>]*>)?", n).group(0)
        print(f"{k:24s} calls {r['Calls']:>4s} avg_us {float(r['AverageNs']) / 1e3:8.2f}")
PY
