# same-box A/B of the lane kernels at C4: HEAD library (contiguous chunks only) vs the tree
set -u
export TMPDIR=/tmp
SHADOW_GPU_LIB=$PWD/tools/ab/libshadow_gpu_head.so bash tools/lane_stats.sh r05c_head || exit 1
bash tools/lane_stats.sh r05c_new || exit 1
SHADOW_GPU_LIB=$PWD/tools/ab/libshadow_gpu_head.so bash tools/lane_stats.sh r05c_head2 || exit 1
bash tools/lane_stats.sh r05c_new2 || exit 1
