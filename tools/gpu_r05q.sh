# C5 lane diag with the slowest block named
set -u
export TMPDIR=/tmp
C5DIAG_OUT=r05q_c5 bash tools/gpu_c5diag.sh
