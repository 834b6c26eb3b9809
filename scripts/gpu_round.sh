#!/bin/bash
# Round-end style session: all GPU tests, smoke, headline bench (1 GPU), kernel-trace profile and
# per-kernel PMC counters of the bench step. Every GPU step has its own time limit; the chain stops
# at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/r_pytest.log 2>&1 && \
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/r_smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r_bench.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --batch-per-gpu 128 > gpurun_out/r_bench128.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r_prof -o run -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/r_prof.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE SQ_INSTS_MFMA --output-format csv -d gpurun_out/r_pmc1 -o pmc -- python3 bench.py --steps 3 --warmup 1 > gpurun_out/r_pmc1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INST_LEVEL_VMEM --output-format csv -d gpurun_out/r_pmc2 -o pmc -- python3 bench.py --steps 3 --warmup 1 > gpurun_out/r_pmc2.log 2>&1
rc=$?
tail -2 gpurun_out/r_pytest.log; tail -1 gpurun_out/r_smoke.log; tail -1 gpurun_out/r_bench.log | cut -c1-250; tail -1 gpurun_out/r_bench128.log | cut -c1-250
exit $rc
