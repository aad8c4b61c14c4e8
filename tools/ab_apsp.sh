#!/bin/bash
# A/B of APSP variants with the v1 library as an in-run control (same box, same process order).
# usage: bash tools/ab_apsp.sh "w64,64,32f" [extra env assignments for the variant run]
export TMPDIR=/tmp
V=${1:-w64}
shift
timeout -k 10 150 env SHADOW_GPU_LIB=tools/ab/libshadow_gpu_v1.so python tools/apsp_variants.py --variants 64 2>&1 | grep variant | sed 's/^/[v1 control] /'
timeout -k 10 300 env "$@" python tools/apsp_variants.py --variants $V 2>&1 | grep variant
timeout -k 10 150 env SHADOW_GPU_LIB=tools/ab/libshadow_gpu_v1.so python tools/apsp_variants.py --variants 64 2>&1 | grep variant | sed 's/^/[v1 control] /'
