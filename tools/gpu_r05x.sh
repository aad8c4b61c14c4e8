# N = 8 rank block (rows 0:1250 of C3) plan knobs (tools/sssp_ab.py --rows, tables compared bit for bit)
set -u
export TMPDIR=/tmp
O=gpurun_out/r05x; mkdir -p $O
timeout -k 10 400 python3 -u tools/sssp_ab.py --reps 9 --rows 0:1250 "" "SG_SSSP_PHASES=3" "SG_SSSP_PHASES=4" "SG_SSSP_BOUNDS=3" "SG_SSSP_BOUNDS=4" "SG_SSSP_FLAGGED=0" "SG_SSSP_HOPS=1" "" > $O/ab.log 2>&1; grep setting $O/ab.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['setting'] or 'default', d['ms_median'], d['ms_min'], d['same_as_first'])"
