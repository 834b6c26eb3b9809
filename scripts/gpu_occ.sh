#!/bin/bash
# Occupancy probe of the conv1 Winograd GEMM: cfg 4 (4 of 9 outputs, 40 KiB ring, up to 4 WG/CU) vs
# cfg 5 (same work, 80 KiB ring, 2 WG/CU) vs cfg 1 (all 9 outputs, 2 WG/CU). Results of 4/5 are wrong.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 1 4 5; do
  ANX_CONV1_WINO_CFG=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/occ_$v -o run -- python3 tools/sweep_batch.py --batches 300 --rounds 2 --iters 5 > gpurun_out/occ_$v.log 2>&1 || exit $?
done
for v in 1 4 5; do echo "cfg $v"; python3 tools/rocprof_summary.py gpurun_out/occ_$v/run_results.db | grep -E "conv1_wino_gemm"; done
