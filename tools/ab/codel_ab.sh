#!/bin/bash
# CoDel leg A/B per library: ops/s and the kernel's average launch.
for lib in "$@"; do
  SHADOW_GPU_LIB=$lib timeout -k 10 200 python bench.py --no-cpu --steps 10 2>/dev/null | grep metric > /tmp/ab.json
  python3 -c "
import json,sys; d=json.load(open('/tmp/ab.json'))['codel']
print(sys.argv[1], d['value'], d['ms_per_batch'], d['roofline']['avg_launch_ms'])" $lib
done
