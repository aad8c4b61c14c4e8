set -u
O=gpurun_out/r8y; mkdir -p $O
for l in g1 g3 g4; do [ -f tools/ab/libshadow_gpu_$l.so ] || { echo missing $l; exit 1; }; done
for r in 0 1; do
  for l in base g1 g3 g4; do
    if [ $l = base ]; then L=shadow_amd/libshadow_gpu.so; else L=tools/ab/libshadow_gpu_$l.so; fi
    SHADOW_GPU_LIB=$L timeout -k 10 300 python3 -u tools/apsp_c2.py --variants "SG_APSP_B=64" --reps 9 --rounds 3 > $O/$l$r.log 2>&1 || { tail -20 $O/$l$r.log; exit 1; }
    echo "$l: $(grep -v amdgpu $O/$l$r.log | grep ms/build | tr '\n' ' ')"
  done
done
