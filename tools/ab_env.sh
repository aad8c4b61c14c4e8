# A/B of environment settings on the bench line (separate processes, alternated).
# usage: bash tools/ab_env.sh OUT REPS "ENV1" "ENV2" ...   ("-" = no extra environment)
set -u
OUT=$1; REPS=$2; shift 2
mkdir -p $(dirname $OUT)
for r in $(seq $REPS); do
  for e in "$@"; do
    if [ "$e" = "-" ]; then envs=""; else envs="$e"; fi
    env $envs timeout -k 10 300 python3 bench.py --no-cpu --no-gml --no-c2 --rank-blocks 8 --steps 10 2>/dev/null | grep metric > /tmp/ab_env.json || { echo "run failed: $e"; exit 1; }
    python3 - "$e" >> $OUT << 'PY'
import json, sys
d = json.load(open("/tmp/ab_env.json"))
dl, ib, ob, cd = d["delivery"], d["inbound"], d["outbound"], d["codel"]
print(f"{sys.argv[1]:30s} c3 {d['ms_per_step']:.4f} rb8 {d['apsp_detail']['rank_block_ms']['8']['max_ms']:.4f} "
      f"c4 {dl['ms_per_round']:.4f} codel {cd.get('ms_per_batch')} inb {ib.get('ms_per_window')} outb {ob.get('ms_per_window')}")
PY
  done
done
cat $OUT
