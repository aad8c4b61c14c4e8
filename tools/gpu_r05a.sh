# lane-major chunks (k_codel): codel tests, C4 lane stats, C5 lane diag
set -u
O=gpurun_out/r05a; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_codel_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/lane_stats.sh r05a || exit 1
bash tools/gpu_c5diag.sh || exit 1
