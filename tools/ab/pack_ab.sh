#!/bin/bash
# Delivery A/B: two-array table vs packed path-key table, alternated.
set -o pipefail
for i in 1 2; do
  for flag in --no-pack ""; do
    timeout -k 10 200 python bench.py --no-cpu --steps 20 $flag 2>/dev/null | grep metric > /tmp/ab.json || exit 1
    python3 -c "
import json,sys; d=json.load(open('/tmp/ab.json'))['delivery']
print(sys.argv[1] or 'packed', d['ms_per_round'], d['table_pack_ms'], d['roofline']['achieved'], d['kernel_ms'])" "$flag"
  done
done
