# C4 lane diag: HEAD library vs the tree (block and walk times of the lane kernels)
set -u
O=gpurun_out/r05f; mkdir -p $O
export TMPDIR=/tmp
run() {  # $1 = name; the rest: env assignments
  local v=$1; shift
  env "$@" SG_LANE_DIAG=1 timeout -k 10 300 python3 -u bench.py --no-cpu --no-gml --no-c2 --no-compare --steps 1 --warmup 0 --rank-blocks '' > $O/$v.json 2> $O/$v.err || { tail -5 $O/$v.err; return 1; }
  echo "== $v"; for k in k_codel k_inbound k_outbound; do grep "\[lane\] $k" $O/$v.err | tail -2; done
}
run head SHADOW_GPU_LIB=$PWD/tools/ab/libshadow_gpu_head.so && run new SG_X=0
