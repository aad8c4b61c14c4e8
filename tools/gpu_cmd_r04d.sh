set -u
O=gpurun_out/r04d; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest tests/test_routing_gpu.py tests/test_routing_fuzz_gpu.py tests/test_deliver_gpu.py tests/test_dist_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/sssp_ab.py --reps 7 SG_SSSP_FLAGGED=0 SG_SSSP_FLAGGED=1 SG_SSSP_FLAGGED=1,SG_SSSP_PHASES=2 SG_SSSP_FLAGGED=1,SG_SSSP_PHASES=4 > $O/ab_full.log 2>&1 || exit 1
for R in 8750:10000 7500:10000 5000:10000; do
  timeout -k 10 200 python3 tools/sssp_ab.py --reps 9 --rows $R SG_SSSP_FLAGGED=0 SG_SSSP_FLAGGED=1 SG_SSSP_FLAGGED=1,SG_SSSP_PHASES=3 SG_SSSP_FLAGGED=1,SG_SSSP_BOUNDS=3 > $O/ab_rows_${R/:/_}.log 2>&1 || exit 1
done
cat $O/ab_*.log | cut -c1-200
for L in tools/ab/libshadow_gpu_r03.so ""; do
  export SHADOW_GPU_LIB=$L; [ -z "$L" ] && unset SHADOW_GPU_LIB
  echo "lib=${L:-new}"
  timeout -k 10 200 python3 tools/round_c5.py --rounds 30 --nodes 10000 --hosts 100000 --packets 1000000 2>&1 | tail -2 || exit 1
  timeout -k 10 200 python3 tools/round_c5.py --rounds 8 2>&1 | tail -2 || exit 1
done
unset SHADOW_GPU_LIB
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2prof -o run -- python3 tools/apsp_c2.py --variants "SG_APSP_DENSE=1" --reps 5 --rounds 2 > $O/c2prof.log 2>&1 || exit 1
find $O/c2prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_c2.csv \;
echo done
