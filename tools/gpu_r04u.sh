# A/B of the explicit ring-path wait in Q::load_head: lane tests, then lane kernel stats.
set -u
O=gpurun_out/r04u; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_codel_gpu.py tests/test_inbound_gpu.py tests/test_outbound_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/lane_stats.sh r04u || exit 1
bash tools/lane_stats.sh r04u2 || exit 1
