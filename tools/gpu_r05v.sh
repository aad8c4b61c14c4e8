# lane-major walk (k_walk_lm): delivery + C5 tests, C4 round A/B vs HEAD, C5 round timing
set -u
O=gpurun_out/r05v; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_deliver_gpu.py tests/test_c5_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
SHADOW_GPU_LIB=$PWD/tools/ab/libshadow_gpu_head.so timeout -k 10 120 python3 -u tools/round_c4.py "" > $O/c4_head.log 2>&1 && grep round $O/c4_head.log
timeout -k 10 120 python3 -u tools/round_c4.py "" > $O/c4_new.log 2>&1 && grep round $O/c4_new.log
SG_LANE_MAJOR=0 timeout -k 10 300 python3 -u tools/round_c5.py > $O/c5_contig.log 2>&1 && tail -2 $O/c5_contig.log
timeout -k 10 300 python3 -u tools/round_c5.py > $O/c5_lm.log 2>&1 && tail -2 $O/c5_lm.log
