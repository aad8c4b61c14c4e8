#!/bin/bash
# PMC passes over the LDS-resident search kernel (one C3 build, k_sssp_lds only).
# usage (GPU box): bash tools/pmc_sssp.sh TAG
set -u
TAG=${1:-x}
export TMPDIR=/tmp
OUT=gpurun_out/pmc_sssp_$TAG
mkdir -p $OUT
run() {  # name counters...
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --kernel-include-regex k_sssp_lds --pmc "$@" --output-format csv -d $OUT/$name -o run -- python3 tools/sssp_one.py > $OUT/$name.log 2>&1 || { echo "pass $name failed"; tail -5 $OUT/$name.log; exit 1; }
}
run sq1 SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS
run sq2 SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_ANY
run tcc TCC_HIT_sum TCC_MISS_sum
run tcp TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum
run ta TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum
run grbm GRBM_GUI_ACTIVE GRBM_COUNT
echo pmc done
