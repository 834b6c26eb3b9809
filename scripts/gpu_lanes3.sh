#!/bin/bash
# bench.py over images per GPU x lanes at whole-wave batch sizes (300 images per lane fills waves).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
for cfg in "600 2" "1200 2" "1200 4" "600 4" "1200 3" "600 2"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 --batch-per-gpu $1 --lanes $2 > gpurun_out/l3_$1_$2_$r.log 2>&1 || exit $?
  echo "B $1 lanes $2: $(grep '"metric"' gpurun_out/l3_$1_$2_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
done
