set -u
O=gpurun_out/r7p; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_deliver_gpu.py tests/test_dist_gpu.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 300 python3 -u tools/round_c4.py "" > $O/r.log 2>&1; grep -v amdgpu $O/r.log | tail -2
