#!/bin/bash
# Kernel trace of the unfused path (fuse_pool1=0: pool1 kernel + plain transform) next to the fused one,
# one lane at 128 images.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r03_pt -o run -- python3 tools/ab_variants.py \
  --arms "fuse_pool1=0|fuse_pool1=1" --batch 128 --rounds 3 > gpurun_out/r03_pt.log 2>&1
