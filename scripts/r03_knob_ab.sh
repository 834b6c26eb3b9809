#!/bin/bash
# Knob A/B (currently conv1_band): GPU engine + Winograd numerics tests, in-process A/B, bench A/B (alternating arms), kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
O=gpurun_out/r03_fuse
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -x -q -k band --timeout 120 --timeout-method thread > $O.tests.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/ab_variants.py --arms "conv1_band=0|conv1_band=1|conv1_band=2" --batch 128 --lanes 1 --rounds 5 > $O.ab.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/ab_variants.py --arms "conv1_band=0|conv1_band=1|conv1_band=2" --batch 300 --lanes 1 --rounds 5 >> $O.ab.log 2>&1 || exit $?
for r in 1 2 3; do
  for f in 1 2; do
    timeout -k 10 200 python -u bench.py --steps 200 --warmup 10 --no-b1 --knob conv1_band=$f >> $O.bench.jsonl 2>> $O.err || exit $?
  done
done
for f in 1 2; do
  timeout -k 10 200 python -u bench.py --batch-per-gpu 64 --steps 200 --warmup 10 --no-b1 --knob conv1_band=$f >> $O.bench.jsonl 2>> $O.err || exit $?
done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_fuse" -o run -- \
  python3 "$GRAFT_REPO_ROOT/tools/ab_variants.py" --arms "conv1_band=0|conv1_band=1|conv1_band=2" --batch 128 --rounds 2 > "$GRAFT_REPO_ROOT/$O.prof.log" 2>&1
