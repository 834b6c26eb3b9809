#!/bin/bash
# A/B of non-temporal V stores in the two Winograd input transforms (kernel-trace timing).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 0 1; do
  ANX_WINO_PRIO=$((1 + 2 * v)) ANX_CONV1_WINO_PROBE=$((16 + 32 * v)) timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/nt_$v -o run -- python3 tools/sweep_batch.py --batches 300 --rounds 2 --iters 5 > gpurun_out/nt_$v.log 2>&1 || exit $?
done
for v in 0 1; do echo "nt $v"; python3 tools/rocprof_summary.py gpurun_out/nt_$v/run_results.db | grep -E "_in_kernel|wino_fused|conv1_wino_gemm"; grep batch gpurun_out/nt_$v.log; done
