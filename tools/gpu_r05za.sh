# N = 8 rank block (rows 0:1250 of C3): seed hops and bound rows, interleaved repeats
set -u
export TMPDIR=/tmp
O=gpurun_out/r05za; mkdir -p $O
timeout -k 10 500 python3 -u tools/sssp_ab.py --reps 15 --rows 0:1250 "" "SG_SSSP_HOPS=1" "" "SG_SSSP_HOPS=1" "SG_SSSP_BOUNDS=4" "" "SG_SSSP_BOUNDS=4" "SG_SSSP_HOPS=1,SG_SSSP_BOUNDS=4" > $O/ab.log 2>&1; grep setting $O/ab.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['setting'] or 'default', d['ms_median'], d['ms_min'], d['same_as_first'])"
