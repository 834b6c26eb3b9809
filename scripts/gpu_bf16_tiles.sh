#!/bin/bash
# A/B: full AlexNet bf16 at 256 images with conv3-5 on 128x128 (default) vs 64x64 tiles.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  for mk in 4194304 20000000 12000000; do
    ANX_BF16_SMALL_MK=$mk timeout -k 10 300 python bench.py --model full --batch-per-gpu 256 --steps 30 --warmup 5 > gpurun_out/bt_${mk}_$r.log 2>&1 || exit $?
    echo "small_mk $mk round $r: $(grep '"metric"' gpurun_out/bt_${mk}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
