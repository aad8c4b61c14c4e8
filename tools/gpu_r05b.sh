# lane-major chunks in k_codel / k_inbound / k_outbound: lane tests, C4 lane stats, C5 lane diag
set -u
O=gpurun_out/r05b; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_codel_gpu.py tests/test_inbound_gpu.py tests/test_outbound_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/lane_stats.sh r05b || exit 1
C5DIAG_OUT=r05b_c5 bash tools/gpu_c5diag.sh || exit 1
