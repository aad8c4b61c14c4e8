set -u
O=gpurun_out/r8r; mkdir -p $O
[ -f tools/ab/libshadow_gpu_head.so ] || { echo missing lib; exit 1; }
timeout -k 10 600 python3 -u -m pytest tests/test_outbound_gpu.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for r in 0 1; do
  for l in head new; do
    if [ $l = new ]; then L=shadow_amd/libshadow_gpu.so; else L=tools/ab/libshadow_gpu_$l.so; fi
    SHADOW_GPU_LIB=$L timeout -k 10 300 python3 -u bench.py --no-cpu --no-gml --no-c2 --no-compare --steps 3 --rank-blocks "" > $O/b_$l$r.json 2> $O/b_$l$r.err || { tail -5 $O/b_$l$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/b_$l$r.json').read().strip().splitlines()[-1]); o=d['outbound']; print('$l', o['ms_per_window'], o['roofline'].get('avg_launch_ms'), o.get('compact_ms'))"
  done
done
