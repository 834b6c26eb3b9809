#!/bin/bash
# Lanes x Winograd tail split A/B at the bench default batch (one box, interleaved): writes
# gpurun_out/ab_lanes.txt. usage: bash scripts/ab_lanes.sh [BATCH]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
B=${1:-128}
for rep in 1 2; do
  for lanes in 1 2 3 4; do
    for split in 0 1; do
      v=$(ANX_WINO_SPLIT=$split timeout -k 10 120 python bench.py --steps 30 --warmup 5 --lanes $lanes --batch-per-gpu $B 2>/dev/null | grep -o '"value": [0-9.]*') || exit 1
      echo "batch=$B lanes=$lanes split=$split $v" | tee -a gpurun_out/ab_lanes.txt
    done
  done
done
