set -u
O=gpurun_out/r8i; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_routing_gpu.py tests/test_routing_fuzz_gpu.py -x -q --timeout 300 --timeout-method thread -k "bucket or band_degree" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
export SG_BUCKET_DIAG=1
V="SG_APSP_BUCKET=1;SG_APSP_BUCKET=1 SG_BAND_PREFETCH=0"
timeout -k 10 400 python3 -u tools/apsp_ab.py --rows 12800 --rounds 2 --variants "$V" > $O/ab.log 2>&1 || { tail -30 $O/ab.log; exit 1; }
grep -E "median|identical|DIFF|wave 0|phase 0" $O/ab.log
