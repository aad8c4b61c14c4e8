set -u
O=gpurun_out/r8v; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_routing_gpu.py tests/test_routing_fuzz_gpu.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 300 python3 -u tools/apsp_c2.py --variants "SG_APSP_B=64;SG_DENSE_SPLIT=0" --reps 9 --rounds 3 > $O/c2.log 2>&1 || { tail -20 $O/c2.log; exit 1; }
grep -v amdgpu $O/c2.log | tail -4
