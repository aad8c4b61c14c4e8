# lane-major chunks only in launches that can use them (ANY): lane tests, same-box C4 A/B vs HEAD, C5 diag
set -u
O=gpurun_out/r05e; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_codel_gpu.py tests/test_inbound_gpu.py tests/test_outbound_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
SHADOW_GPU_LIB=$PWD/tools/ab/libshadow_gpu_head.so bash tools/lane_stats.sh r05e_head || exit 1
bash tools/lane_stats.sh r05e_new || exit 1
C5DIAG_OUT=r05e_c5 bash tools/gpu_c5diag.sh || exit 1
