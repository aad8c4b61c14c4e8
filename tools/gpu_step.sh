set -u
O=gpurun_out/r8l; mkdir -p $O
[ -f tools/ab/libshadow_gpu_head.so ] || { echo missing lib; exit 1; }
timeout -k 10 600 python3 -u -m pytest tests/test_routing_gpu.py tests/test_routing_fuzz_gpu.py -x -q --timeout 300 --timeout-method thread -k "bucket or band_degree" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for r in 0 1; do
  for l in head new; do
    if [ $l = new ]; then L=shadow_amd/libshadow_gpu.so; else L=tools/ab/libshadow_gpu_$l.so; fi
    SHADOW_GPU_LIB=$L timeout -k 10 300 python3 -u tools/apsp_ab.py --rows 12800 --rounds 2 --variants "SG_APSP_BUCKET=1" > $O/$l$r.log 2>&1 || { tail -30 $O/$l$r.log; exit 1; }
    echo "$l: $(grep median $O/$l$r.log)"
  done
done
SG_BUCKET_DIAG=1 timeout -k 10 300 python3 -u tools/apsp_ab.py --rows 12800 --rounds 1 --variants "SG_APSP_BUCKET=1" > $O/diag.log 2>&1 || { tail -30 $O/diag.log; exit 1; }
grep -E "bucket\]" $O/diag.log
