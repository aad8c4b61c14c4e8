# Plan kernels of the tree's library against the previous one (tools/ab/build_rev.sh HEAD prev): the
# routing tests, kernel-trace averages of one-shot C3 builds, then an interleaved one-shot A/B.
set -u
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_routing_gpu.py \
  tests/test_routing_options_gpu.py -m gpu > gpurun_out/plan_tests.txt 2>&1 || { tail -5 gpurun_out/plan_tests.txt; exit 1; }
tail -1 gpurun_out/plan_tests.txt
for lib in tools/ab/libshadow_gpu_prev.so shadow_amd/libshadow_gpu.so; do
  SHADOW_GPU_LIB=$PWD/$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv \
    -d gpurun_out/plan_prof_$(basename $lib .so) -o run -- python3 tools/oneshot_parts.py 10000 > /dev/null 2>&1 || exit 1
done
timeout -k 10 500 bash tools/ab/oneshot_lib_ab.sh > gpurun_out/ab_plan.txt 2>&1 || exit 1
