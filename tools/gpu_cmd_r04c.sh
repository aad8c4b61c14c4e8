set -u
mkdir -p gpurun_out/r04c
timeout -k 10 400 python3 -u -m pytest tests/test_deliver_gpu.py tests/test_dist_gpu.py tests/test_routing_gpu.py tests/test_routing_fuzz_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r04c/tests.log 2>&1; rc=$?; tail -3 gpurun_out/r04c/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 tools/apsp_c2.py --variants "SG_APSP_DENSE=0;SG_APSP_DENSE=1" --reps 5 --rounds 3 > gpurun_out/r04c/c2.log 2>&1; rc=$?; tail -4 gpurun_out/r04c/c2.log; [ $rc -eq 0 ] || exit $rc
for L in tools/ab/libshadow_gpu_r03.so ""; do
  export SHADOW_GPU_LIB=$L; [ -z "$L" ] && unset SHADOW_GPU_LIB
  echo "lib=${L:-new}"
  timeout -k 10 200 python3 tools/round_c5.py --rounds 30 --nodes 10000 --hosts 100000 --packets 1000000 2>&1 | tail -3 || exit 1
  timeout -k 10 200 python3 tools/round_c5.py --rounds 8 2>&1 | tail -3 || exit 1
done
unset SHADOW_GPU_LIB
bash tools/prof_rounds.sh r04c_new && bash tools/prof_rounds.sh r04c_r03 tools/ab/libshadow_gpu_r03.so
