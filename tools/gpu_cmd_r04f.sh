set -u
O=gpurun_out/r04f; mkdir -p $O
export TMPDIR=/tmp
SG_SORT_DIAG=1 timeout -k 10 200 python3 tools/round_c5.py --rounds 3 --nodes 10000 --hosts 100000 --packets 1000000 > $O/sortdiag_c4.log 2>&1 || exit 1
SG_SORT_DIAG=1 timeout -k 10 200 python3 tools/round_c5.py --rounds 3 > $O/sortdiag_c5.log 2>&1 || exit 1
grep "\[sort\]" $O/sortdiag_c4.log | tail -2; grep "\[sort\]" $O/sortdiag_c5.log | tail -2
timeout -k 10 300 python3 -u -m pytest tests/test_routing_gpu.py tests/test_routing_fuzz_gpu.py tests/test_routing_options_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread -k "dense or complete or c2 or random_graph_shapes or direct or option" > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 tools/apsp_c2.py --variants "SG_APSP_DENSE=1" --reps 5 --rounds 3 > $O/c2.log 2>&1; rc=$?; tail -2 $O/c2.log; [ $rc -eq 0 ] || exit $rc
bash tools/pmc_sssp.sh r04f > $O/pmc_sssp.log 2>&1 || { tail -5 $O/pmc_sssp.log; exit 1; }
bash tools/pmc_kernel.sh r04f_c5 "k_sb_sort_region,k_walk,k_sb_scatter" python3 tools/round_c5.py --rounds 2 > $O/pmc_c5.log 2>&1 || { tail -5 $O/pmc_c5.log; exit 1; }
tail -60 $O/pmc_c5.log
echo done
