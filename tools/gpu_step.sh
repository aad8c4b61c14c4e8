set -u
O=gpurun_out/r6w; mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests/test_routing_gpu.py -x -q --timeout 200 --timeout-method thread -k "c3_full_table or random_sparse or row_blocks or persistent or variants" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for r in 1 2 3; do
  for L in tools/ab/base_r6.so shadow_amd/libshadow_gpu.so; do
    SHADOW_GPU_LIB=$PWD/$L timeout -k 10 120 python3 -u tools/apsp_ab.py --nodes 10000 --variants "SG_SSSP_X=0" --reps 7 --rounds 1 > $O/ab_$r.log 2>&1 || { tail $O/ab_$r.log; exit 1; }
    echo "$L $(grep median $O/ab_$r.log | sed 's/; sssp.*//')"
  done
done
