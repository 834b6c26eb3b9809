#!/bin/bash
# PMC passes over the default bench.py step (600 images as 2 stream lanes); kernel-trace only.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU --output-format csv -d gpurun_out/pl1 -o pmc -- python3 bench.py --steps 4 --warmup 2 > gpurun_out/pl1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_INSTS_SALU SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/pl2 -o pmc -- python3 bench.py --steps 4 --warmup 2 > gpurun_out/pl2.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pl3 -o pmc -- python3 bench.py --steps 4 --warmup 2 > gpurun_out/pl3.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pl4 -o pmc -- python3 bench.py --steps 4 --warmup 2 > gpurun_out/pl4.log 2>&1
