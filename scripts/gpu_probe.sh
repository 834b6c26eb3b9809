#!/bin/bash
# Cost probes of the conv1 Winograd GEMM (skip fold / skip DMA refills): one kernel-trace run each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for p in ${PROBES:-0 1 2 3}; do
  ANX_CONV1_WINO_PROBE=$p timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/probe_$p -o run -- python3 tools/sweep_batch.py --batches 300 --rounds 1 --iters 4 > gpurun_out/probe_$p.log 2>&1 || exit $?
done
for p in ${PROBES:-0 1 2 3}; do echo "probe $p"; python3 tools/rocprof_summary.py gpurun_out/probe_$p/run_results.db | grep -E "conv1_wino|wino_fused"; done
