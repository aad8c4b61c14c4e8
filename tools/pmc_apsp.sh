#!/bin/bash
# PMC passes over APSP builds (kernel k_relax<...>), for diagnosis.
# usage: bash tools/pmc_apsp.sh TAG ["ENV=VAL ENV2=VAL2"]   (one variant, see tools/apsp_variants.py)
set -u
TAG=$1
VAR=${2:-}
export TMPDIR=/tmp
OUT=gpurun_out/pmc_$TAG; mkdir -p $OUT
run() { name=$1; shift; timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o run -- python3 tools/apsp_variants.py --reps 1 --variants "$VAR" > $OUT/$name.log 2>&1 || echo "pass $name failed"; }
run sq SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU
run lvl SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS
run tcc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE
run fetch FETCH_SIZE
run tcp TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum
python3 - "$OUT" "${KFILTER:-k_relax_w2<}" <<'PY'
import csv, glob, sys, collections
out, kf = sys.argv[1], sys.argv[2]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(lambda: collections.defaultdict(int))
for f in glob.glob(out + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if kf not in k:
            continue
        acc["k_relax"][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt["k_relax"][r["Counter_Name"]] += 1
for k, d in acc.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:30s} total {v:14.4g}  per-dispatch {v / cnt[k][c]:14.4g}")
PY
