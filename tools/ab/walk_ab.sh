#!/bin/bash
# Delivery-kernel A/B: per-kernel ms of one C4 round for each library given.
for lib in "$@"; do
  SHADOW_GPU_LIB=$lib timeout -k 10 200 python bench.py --no-cpu --steps 10 2>/dev/null | grep metric > /tmp/ab.json
  python3 -c "
import json,sys; d=json.load(open('/tmp/ab.json'))['delivery']; print(sys.argv[1], d['ms_per_round'], d['kernel_ms'])" $lib
done
