set -u
O=gpurun_out/r04q; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_codel_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/lane_stats.sh r04q || exit 1
SG_LANE_DIAG=1 timeout -k 10 150 python3 bench.py --no-cpu --no-gml --no-c2 --no-compare --rank-blocks= --steps 1 --warmup 0 > /dev/null 2> $O/diag.err || exit 1
grep "\[lane\]" $O/diag.err | head -3
