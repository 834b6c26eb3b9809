#!/bin/bash
# Conv1 band transform: 2 phase rows per workgroup (conv1_band=1) vs 4 phase rows x half the tile
# columns (=2, every 192-B V row segment written whole by one workgroup): bitwise tests, kernel trace
# of one lane, bench step alternating arms.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out/r03_bs
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -x -q -k band --timeout 120 --timeout-method thread > $O.tests.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O.prof -o run -- python3 tools/ab_variants.py \
  --arms "conv1_band=1|conv1_band=2" --batch 128 --rounds 3 > $O.ab.log 2>&1 || exit $?
for r in 1 2; do
  for f in 1 2; do
    timeout -k 10 200 python -u bench.py --steps 200 --warmup 10 --no-b1 --knob conv1_band=$f >> $O.bench.jsonl 2>> $O.err || exit $?
  done
done
