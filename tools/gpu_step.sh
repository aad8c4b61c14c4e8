set -u
O=gpurun_out/r8q; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_routing_gpu.py tests/test_routing_fuzz_gpu.py -x -q --timeout 300 --timeout-method thread -k "bucket or band" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
SG_BAND_PAIR=1 timeout -k 10 600 python3 -u -m pytest tests/test_routing_gpu.py tests/test_routing_fuzz_gpu.py -x -q --timeout 300 --timeout-method thread -k "bucket or band" > $O/tp.log 2>&1 || { tail -30 $O/tp.log; exit 1; }
tail -1 $O/tp.log
SG_BAND_PAIR=1 timeout -k 10 600 python3 -u -m pytest tests/test_c5_gpu.py -x -q --timeout 500 --timeout-method thread > $O/t5.log 2>&1 || { tail -30 $O/t5.log; exit 1; }
tail -1 $O/t5.log
export SG_BUCKET_DIAG=1
timeout -k 10 400 python3 -u tools/apsp_ab.py --rows 12800 --rounds 2 --variants "SG_APSP_BUCKET=1;SG_APSP_BUCKET=1 SG_BAND_PAIR=1" > $O/ab.log 2>&1 || { tail -30 $O/ab.log; exit 1; }
grep -E "median|identical|DIFF|bucket\]" $O/ab.log
