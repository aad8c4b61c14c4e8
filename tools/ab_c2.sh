# A/B of environment settings on the C2 leg of the bench line (separate processes, alternated).
# usage: bash tools/ab_c2.sh OUT REPS "ENV1" "ENV2" ...   ("-" = no extra environment)
set -u
OUT=$1; REPS=$2; shift 2
mkdir -p $(dirname $OUT)
for r in $(seq $REPS); do
  for e in "$@"; do
    if [ "$e" = "-" ]; then envs=""; else envs="$e"; fi
    env $envs timeout -k 10 300 python3 bench.py --no-cpu --no-gml --no-delivery --no-codel --no-compare --no-e2e \
      --rank-blocks "" --steps 20 2>/dev/null | grep metric > /tmp/ab_c2.json || { echo "run failed: $e"; exit 1; }
    python3 - "$e" >> $OUT << 'PY'
import json, sys
d = json.load(open("/tmp/ab_c2.json"))["c2"]
r = d["roofline"] or {}
print(f"{sys.argv[1]:24s} c2 {d['value'] * 1e3:.4f} ms  one_shot {d['one_shot_s'] * 1e3:.4f} ms  "
      f"launch {r.get('avg_launch_ms')} ms  rel/launch {r.get('relaxations_per_launch')}")
PY
  done
done
cat $OUT
