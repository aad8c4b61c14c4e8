# C2 leg A/B of two libraries, alternated: bash tools/ab/c2_lib_ab.sh OUT REPS LIB_A LIB_B
set -u
OUT=$1; REPS=$2; A=$3; B=$4
for r in $(seq $REPS); do
  for lib in $A $B; do
    SHADOW_GPU_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --no-cpu --no-gml --no-delivery --no-codel --no-compare \
      --no-e2e --rank-blocks= --steps 20 2>/dev/null | grep metric > /tmp/ab_c2l.json || { echo "run failed: $lib"; exit 1; }
    python3 -c "
import json,sys; d=json.load(open('/tmp/ab_c2l.json'))['c2']; r=d['roofline'] or {}
print(f\"{sys.argv[1]:40s} c2 {d['value']*1e3:.4f} ms one_shot {d['one_shot_s']*1e3:.4f} ms sort {r.get('arc_sort_ms')} launch {r.get('avg_launch_ms')} rel {r.get('relaxations_per_launch')}\")" $lib >> $OUT
  done
done
cat $OUT
