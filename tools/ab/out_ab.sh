#!/bin/bash
# APSP A/B per library: build ms and the out-kernel ms (bench timers).
for lib in "$@"; do
  SHADOW_GPU_LIB=$lib timeout -k 10 200 python bench.py --no-cpu --no-delivery --steps 5 2>/dev/null | grep metric > /tmp/ab.json
  python3 -c "
import json,sys; d=json.load(open('/tmp/ab.json'))
print(sys.argv[1], d['ms_per_step'], 'out', d['apsp_detail']['out_kernel_ms'], d['apsp_detail']['out_kernel_GBs'])" $lib
done
