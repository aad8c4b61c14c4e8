set -u
O=gpurun_out/r04g; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest tests/test_routing_gpu.py tests/test_routing_fuzz_gpu.py tests/test_deliver_gpu.py tests/test_dist_gpu.py tests/test_c5_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
SG_SORT_DIAG=1 timeout -k 10 200 python3 tools/round_c5.py --rounds 3 --nodes 10000 --hosts 100000 --packets 1000000 > $O/sortdiag_c4.log 2>&1 || exit 1
SG_SORT_DIAG=1 timeout -k 10 200 python3 tools/round_c5.py --rounds 3 > $O/sortdiag_c5.log 2>&1 || exit 1
grep "\[sort\]" $O/sortdiag_c4.log | tail -1; grep "\[sort\]" $O/sortdiag_c5.log | tail -1
for L in tools/ab/libshadow_gpu_r03.so ""; do
  export SHADOW_GPU_LIB=$L; [ -z "$L" ] && unset SHADOW_GPU_LIB
  echo "lib=${L:-new}"
  timeout -k 10 200 python3 tools/round_c5.py --rounds 30 --nodes 10000 --hosts 100000 --packets 1000000 2>&1 | tail -1 || exit 1
  timeout -k 10 200 python3 tools/round_c5.py --rounds 8 2>&1 | tail -1 || exit 1
  timeout -k 10 200 python3 tools/sssp_ab.py --reps 9 SG_SSSP_FLAGGED=0 2>&1 | grep setting | cut -c1-120 || exit 1
done
unset SHADOW_GPU_LIB
echo done
