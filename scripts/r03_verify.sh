#!/bin/bash
# Round-3 verification: every GPU test, smoke, the bench default, a kernel trace of the bench step
# (2 free-running lanes) and per-kernel HBM bytes / clock / MFMA busy (one lane, counter passes).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/v_tests.log 2>&1 || exit $?
timeout -k 10 120 python -u __graft_entry__.py smoke > $O/v_smoke.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py > $O/v_bench.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/v_prof -o run -- python3 bench.py --steps 50 --warmup 5 --no-b1 \
  > $O/v_prof.log 2>&1 || exit $?
BENCH="bench.py --lanes 1 --steps 6 --warmup 2 --no-b1 --prewarm-s 0"
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace \
  --output-format csv -d $O/v_pmc_fetch -o run -- python3 $BENCH > $O/v_pmc_fetch.log 2>&1 &&
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --kernel-trace \
  --output-format csv -d $O/v_pmc_write -o run -- python3 $BENCH > $O/v_pmc_write.log 2>&1 &&
python3 tools/pmc_clock.py $O/v_pmc_fetch $O/v_pmc_write > $O/v_pmc_bytes_b128.md
# lanes 2 / 3 / 4 at 128 images with the joint lane start (200 steps)
for l in 2 3 4; do
  timeout -k 10 200 python -u bench.py --lanes $l --steps 200 --warmup 10 --no-b1 >> $O/v_lanes.jsonl 2>> $O/v_lanes.err || exit $?
done
