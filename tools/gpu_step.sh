set -u
O=gpurun_out/r7r; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_routing_gpu.py tests/test_routing_fuzz_gpu.py -x -q --timeout 300 --timeout-method thread -k "dense or complete or c2 or sorted_arcs" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 120 python3 -u tools/apsp_c2.py --variants "SG_APSP_B=64" --reps 9 --rounds 2 > $O/c2.log 2>&1; grep -v amdgpu $O/c2.log | tail -3
