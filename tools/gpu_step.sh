set -u
O=gpurun_out/r8x; mkdir -p $O
for l in dn512 dn256; do [ -f tools/ab/libshadow_gpu_$l.so ] || { echo missing $l; exit 1; }; done
for r in 0 1; do
  for l in base dn512 dn256; do
    if [ $l = base ]; then L=shadow_amd/libshadow_gpu.so; else L=tools/ab/libshadow_gpu_$l.so; fi
    SHADOW_GPU_LIB=$L timeout -k 10 300 python3 -u tools/apsp_c2.py --variants "SG_APSP_B=64;SG_DENSE_SPLIT=0" --reps 9 --rounds 3 > $O/$l$r.log 2>&1 || { tail -20 $O/$l$r.log; exit 1; }
    echo "$l: $(grep -v amdgpu $O/$l$r.log | grep ms/build | tr '\n' ' ')"
  done
done
SHADOW_GPU_LIB=tools/ab/libshadow_gpu_dn256.so timeout -k 10 600 python3 -u -m pytest tests/test_routing_gpu.py tests/test_routing_fuzz_gpu.py -x -q --timeout 300 --timeout-method thread -k "dense or complete or c2 or sorted_arcs" > $O/t256.log 2>&1 || { tail -30 $O/t256.log; exit 1; }
tail -1 $O/t256.log
