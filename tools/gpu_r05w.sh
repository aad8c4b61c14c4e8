# C3 plan knobs on the final search (tools/sssp_ab.py, one box, tables compared bit for bit)
set -u
export TMPDIR=/tmp
O=gpurun_out/r05w; mkdir -p $O
timeout -k 10 400 python3 -u tools/sssp_ab.py --reps 9 "" "SG_SSSP_FLAGGED=1" "SG_SSSP_FLAGGED=1,SG_SSSP_PHASES=4" "SG_SSSP_FLAGGED=1,SG_SSSP_PHASES=5" "SG_SSSP_PHASES=4" "SG_SSSP_FLAGGED=1,SG_SSSP_BOUNDS=3" "" > $O/ab.log 2>&1; tail -n 12 $O/ab.log
