#!/bin/bash
# bench.py over images per GPU x lanes, and a kernel trace of the 2-lane default.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in "300 2" "600 2" "600 1" "900 3" "512 2" "300 2"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --batch-per-gpu $1 --lanes $2 > gpurun_out/lb_$1_$2.log 2>&1 || exit $?
  echo "B $1 lanes $2: $(tail -1 gpurun_out/lb_$1_$2.log | cut -c100-215)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/lanes_prof -o run -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/lanes_prof.log 2>&1
