set -u
O=gpurun_out/r6m; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_outbound_gpu.py -x -q --timeout 120 --timeout-method thread > $O/outbound.log 2>&1 || { tail -30 $O/outbound.log; exit 1; }
tail -2 $O/outbound.log
timeout -k 10 600 python3 -u tools/apsp_ab.py --nodes 50000 --variants "SG_APSP_BUCKET=0;SG_APSP_BUCKET=1" --reps 1 --rounds 3 > $O/ab.log 2>&1; rc=$?; grep -E "median|round" $O/ab.log; exit $rc
