#!/bin/bash
# PMC passes (one rocprofv3 run per counter group) over a command, summarised per kernel.
# usage: bash tools/pmc_kernel.sh TAG "KERNEL_SUBSTRING[,KERNEL_SUBSTRING...]" python3 bench.py --no-cpu --steps 2
set -u
TAG=$1; KF=$2; shift 2
export TMPDIR=/tmp
OUT=gpurun_out/pmck_$TAG; mkdir -p $OUT
run() { name=$1; shift; timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o run -- "${CMD[@]}" > $OUT/$name.log 2>&1 || echo "pass $name failed"; }
CMD=("$@")
run sq SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU
run lvl SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_INST_LEVEL_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS
run tcc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE
run fetch FETCH_SIZE
run write WRITE_SIZE
python3 - "$OUT" "$KF" <<'PY'
import csv, glob, sys, collections
out, kfs = sys.argv[1], sys.argv[2].split(",")
acc = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(lambda: collections.defaultdict(int))
for f in glob.glob(out + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = next((kf for kf in kfs if kf in r["Kernel_Name"]), None)
        if k is None:
            continue
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[k][r["Counter_Name"]] += 1
for k, d in acc.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:30s} per-dispatch {v / cnt[k][c]:14.4g}")
PY
