#!/bin/bash
# PMC counter run of the engine at batch 128 (kernel-trace only; no sys/runtime trace with --pmc).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU --output-format csv -d gpurun_out/pmc1 -o pmc -- python3 tools/sweep_batch.py --batches 128 --rounds 1 --iters 2 > gpurun_out/pmc1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_INSTS_SALU SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/pmc2 -o pmc -- python3 tools/sweep_batch.py --batches 128 --rounds 1 --iters 2 > gpurun_out/pmc2.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc3 -o pmc -- python3 tools/sweep_batch.py --batches 128 --rounds 1 --iters 2 > gpurun_out/pmc3.log 2>&1
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pmc4 -o pmc -- python3 tools/sweep_batch.py --batches 128 --rounds 1 --iters 2 > gpurun_out/pmc4.log 2>&1
ls -R gpurun_out | head -40
