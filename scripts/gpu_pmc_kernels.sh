#!/bin/bash
# Per-kernel PMC counters of the Blocks 1-2 step at batch 128 (kernel-trace only, no sys/runtime
# traces with --pmc). Each pass is its own rocprofv3 run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name counters...
  local n=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/pmck_$n -o pmc -- \
    python3 bench.py --steps 3 --warmup 1 > gpurun_out/pmck_$n.log 2>&1
}
run 1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE SQ_INSTS_MFMA && \
run 2 SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INST_LEVEL_VMEM && \
run 3 TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TA_DATA_STALLED_BY_TC_CYCLES TCC_HIT_sum TCC_MISS_sum && \
run 4 SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_UNALIGNED_STALL SQ_LEVEL_WAVES SQ_BUSY_CU_CYCLES
rc=$?
python3 tools/pmc_summary.py gpurun_out/pmck_1 gpurun_out/pmck_2 gpurun_out/pmck_3 gpurun_out/pmck_4 > gpurun_out/pmck_summary.md 2>&1
cat gpurun_out/pmck_summary.md | head -60
exit $rc
