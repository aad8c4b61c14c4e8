# Lane-kernel A/B: the lane GPU tests, then two kernel-trace stats runs (tools/lane_stats.sh).
# usage (GPU box): bash tools/gpu_lane_ab.sh TAG
set -u
TAG=$1
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_codel_gpu.py tests/test_inbound_gpu.py tests/test_outbound_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/lane_stats.sh ${TAG}a || exit 1
bash tools/lane_stats.sh ${TAG}b || exit 1
