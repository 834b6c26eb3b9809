#!/bin/bash
# Transform-kernel variants under free-running lanes: conv1_band 1 / 2 x fuse_pool1 1 / 2 (256 / 512 threads;
# earlier: 27 / 14 KiB of LDS), bench step at 128 and 64 images (alternating arms), correctness
# of every arm against arm 0 (ab_variants max_abs_diff_vs_arm0).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
O=gpurun_out/r03_lds
timeout -k 10 300 python -u tools/ab_variants.py --arms "conv1_band=0;fuse_pool1=0|conv1_band=1;fuse_pool1=1|conv1_band=2;fuse_pool1=1|conv1_band=1;fuse_pool1=2|conv1_band=2;fuse_pool1=2" \
  --batch 128 --lanes 1 --rounds 3 > $O.ab.log 2>&1 || exit $?
for b in 128 64; do
  for r in 1 2; do
    for arm in "1 1" "2 1" "1 2" "2 2"; do
      set -- $arm
      timeout -k 10 200 python -u bench.py --batch-per-gpu $b --steps 200 --warmup 10 --no-b1 --knob conv1_band=$1 --knob fuse_pool1=$2 \
        >> $O.bench.jsonl 2>> $O.err || exit $?
    done
  done
done
