# lane-major k_codel with the next chunk's loads in flight: codel tests, C5 codel diag
set -u
O=gpurun_out/r05y; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_codel_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
C5DIAG_OUT=r05y_c5 bash tools/gpu_c5diag.sh || exit 1
