#!/bin/bash
# Per-pass APSP trace for each library given (SG_APSP_TRACE=1), summarised as total ms and per-pass ms.
for lib in "$@"; do
  SHADOW_GPU_LIB=$lib SG_APSP_TRACE=1 timeout -k 10 120 python bench.py --no-delivery --no-cpu --steps 1 --warmup 0 2>&1 \
    | grep "apsp\]" | tail -24 | awk -v L=$lib '{t+=$6; s=s sprintf("%.2f ", $6)} END {printf "%s total %.3f ms: %s\n", L, t, s}'
done
