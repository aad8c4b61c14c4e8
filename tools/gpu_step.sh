set -u
O=gpurun_out/r8p; mkdir -p $O
[ -f tools/ab/libshadow_gpu_head.so ] || { echo missing lib; exit 1; }
timeout -k 10 600 python3 -u -m pytest tests/test_routing_gpu.py tests/test_routing_fuzz_gpu.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for r in 0 1 2; do
  for l in head new; do
    if [ $l = new ]; then L=shadow_amd/libshadow_gpu.so; else L=tools/ab/libshadow_gpu_$l.so; fi
    SHADOW_GPU_LIB=$L timeout -k 10 200 python3 -u tools/oneshot_parts.py 1250 > $O/$l$r.log 2>&1 || { tail -20 $O/$l$r.log; exit 1; }
    echo "$l: $(grep create $O/$l$r.log)"
  done
done
