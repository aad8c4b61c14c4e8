#!/bin/bash
# Kernel-trace stats of delivery rounds alone (no routing build): C4 (10k-node table,
# 100k hosts, 1M packets) and C5 (50k-node table, 10M packets).  On the GPU box:
#   bash tools/prof_rounds.sh TAG [LIB]     (LIB: an A/B library, exported as SHADOW_GPU_LIB)
set -u
TAG=${1:-r}
export TMPDIR=/tmp
[ -n "${2:-}" ] && export SHADOW_GPU_LIB=$2
OUT=gpurun_out/rounds_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c4 -o run -- \
  python3 tools/round_c5.py --rounds 20 --nodes 10000 --hosts 100000 --packets 1000000 > $OUT/c4.log 2>&1 || { echo "c4 failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c5 -o run -- \
  python3 tools/round_c5.py --rounds 10 > $OUT/c5.log 2>&1 || { echo "c5 failed"; exit 1; }
for c in c4 c5; do find $OUT/$c -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats_${c}_$TAG.csv \; ; done
tail -2 $OUT/c4.log $OUT/c5.log
