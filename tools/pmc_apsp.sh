#!/bin/bash
# PMC passes over one APSP build (kernel k_relax_*), for diagnosis.  usage: bash tools/pmc_apsp.sh TAG [env...]
set -u
TAG=$1; shift
export TMPDIR=/tmp
OUT=gpurun_out/pmc_$TAG; mkdir -p $OUT
CMD="python3 tools/apsp_variants.py --variants ${VARIANT:-w64} --reps 1"
run() { name=$1; shift; timeout -k 10 200 env "$ENVS" rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o run -- $CMD > $OUT/$name.log 2>&1 || echo "pass $name failed"; }
ENVS="${1:-X=1}"
run sq SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU
run tcc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE
run fetch FETCH_SIZE
run tcp TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum
run lvl SQ_INSTS_VMEM SQ_INST_LEVEL_VMEM SQ_INSTS_SMEM SQ_INSTS_LDS
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(lambda: collections.defaultdict(int))
for f in glob.glob(out + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "relax" not in k:
            continue
        acc[k[:40]][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[k[:40]][r["Counter_Name"]] += 1
for k, d in acc.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:22s} total {v:14.4g}  per-dispatch {v / cnt[k][c]:14.4g}")
PY
