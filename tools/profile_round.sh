#!/bin/bash
# rocprofv3 evidence for profiles/: kernel-trace stats, then separate PMC passes.
# Usage (on the GPU box): bash tools/profile_round.sh r01 [c3c4|c5|c3|c2]
#   c3: the C3 headline build alone (no delivery, lanes, GML, C2, compare or rank-block builds), so
#       the per-kernel averages are the headline launches'; c2: the C2 leg beside it
set -u
TAG=${1:-r01}
CFG=${2:-c3c4}
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
ARGS="--steps 3 --warmup 1 --no-cpu --no-compare"
[ "$CFG" = c5 ] && ARGS="--config c5 --steps 1 --warmup 1 --no-cpu --no-compare --no-gml --no-c2 --rank-blocks 8"
[ "$CFG" = c3 ] && ARGS="--steps 3 --warmup 1 --no-cpu --no-compare --no-delivery --no-codel --no-gml --no-c2 --no-e2e --rank-blocks="
[ "$CFG" = c2 ] && ARGS="--steps 3 --warmup 1 --no-cpu --no-compare --no-delivery --no-codel --no-gml --no-e2e --rank-blocks="
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python3 bench.py $ARGS > $OUT/stats.log 2>&1 || { echo "stats pass failed"; exit 1; }
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1 || { echo "fetch pass failed"; exit 1; }
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 bench.py $ARGS > $OUT/write.log 2>&1 || { echo "write pass failed"; exit 1; }
timeout -k 10 600 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --output-format csv -d $OUT/sq -o run -- python3 bench.py $ARGS > $OUT/sq.log 2>&1 || { echo "sq pass failed"; exit 1; }
python3 tools/pmc_summary.py --stats $OUT/stats --fetch $OUT/fetch --write $OUT/write --sq $OUT/sq -o $OUT/pmc_$TAG.json > /dev/null
find $OUT -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats_$TAG.csv \;
echo "profile done"
