#!/bin/bash
# PMC passes over one APSP kernel of a tools/apsp_ab.py run (one rocprofv3 run per counter group),
# summarised per dispatch.  usage (GPU box): bash tools/pmc_apsp_kernel.sh TAG KERNEL_REGEX APSP_AB_ARGS...
set -u
TAG=$1; KR=$2; shift 2
export TMPDIR=/tmp
OUT=gpurun_out/pmc_$TAG; mkdir -p $OUT
run() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-include-regex "$KR" --pmc "$@" --output-format csv -d $OUT/$name -o run \
    -- python3 tools/apsp_ab.py "${ARGS[@]}" > $OUT/$name.log 2>&1 || { echo "pass $name failed"; tail -5 $OUT/$name.log; exit 1; }
}
ARGS=("$@")
run sq1 SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS
run sq2 SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_ANY
run tcc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE
run tcp TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_WRITE_REQ_sum
run ta TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum
run fetch FETCH_SIZE
run write WRITE_SIZE
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(out + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:34s} per dispatch (first / last) {v[0]:14.5g} {v[-1]:14.5g}  n={len(v)}")
PY
