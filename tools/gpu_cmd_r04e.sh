set -u
O=gpurun_out/r04e; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_routing_gpu.py tests/test_routing_fuzz_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread -k "dense or complete or c2 or random_graph_shapes or direct" > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 tools/apsp_c2.py --variants "SG_APSP_DENSE=0;SG_APSP_DENSE=1" --reps 5 --rounds 3 > $O/c2.log 2>&1; rc=$?; tail -3 $O/c2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2prof -o run -- python3 tools/apsp_c2.py --variants "SG_APSP_DENSE=1" --reps 5 --rounds 2 > $O/c2prof.log 2>&1 || exit 1
find $O/c2prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_c2.csv \;
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cpu --no-gml --no-compare > $O/bench.json 2> $O/bench.err; rc=$?; tail -c 400 $O/bench.json; [ $rc -eq 0 ] || exit $rc
echo done
