set -u
O=gpurun_out/r9c; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_outbound_gpu.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
