#!/bin/bash
# A/B of s_setprio around the MFMA slices (guide T5) on both Winograd GEMMs, kernel-trace timing.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 0 1; do
  ANX_WINO_PRIO=$v ANX_CONV1_WINO_PROBE=$((16 * v)) timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prio_$v -o run -- python3 tools/sweep_batch.py --batches 300 --rounds 2 --iters 5 > gpurun_out/prio_$v.log 2>&1 || exit $?
done
for v in 0 1; do echo "prio $v"; python3 tools/rocprof_summary.py gpurun_out/prio_$v/run_results.db | grep -E "conv1_wino_gemm|wino_fused"; grep batch gpurun_out/prio_$v.log; done
