#!/bin/bash
# TA / TCP utilisation of one kernel (two PMC passes), e.g. bash tools/pmc_ta.sh "k_relax_w2<" python3 bench.py --no-cpu --no-delivery --steps 1
set -u
KF=$1; shift
export TMPDIR=/tmp
OUT=gpurun_out/pmc_ta; rm -rf $OUT; mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY_sum TA_BUFFER_TOTAL_CYCLES_sum GRBM_GUI_ACTIVE --output-format csv -d $OUT/ta -o run -- "$@" > $OUT/ta.log 2>&1 || echo "ta pass failed"
timeout -s KILL 120 rocprofv3 --pmc TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE --output-format csv -d $OUT/tcp -o run -- "$@" > $OUT/tcp.log 2>&1 || echo "tcp pass failed"
python3 - "$OUT" "$KF" <<'PY'
import csv, glob, sys, collections
out, kf = sys.argv[1], sys.argv[2]
acc = collections.defaultdict(float); cnt = collections.defaultdict(int)
for f in glob.glob(out + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if kf not in r["Kernel_Name"]:
            continue
        acc[r["Counter_Name"]] += float(r["Counter_Value"]); cnt[r["Counter_Name"]] += 1
for c in sorted(acc):
    print(f"{c:40s} per-dispatch {acc[c] / cnt[c]:14.4g}")
PY
