#!/bin/bash
# Test the homework side-track (the reference's scripts/test_hw.sh): homework 1 is the
# row-distributed fp64 DGEMM, here anx_dgemm over anxrun ranks (csrc/src/versions/dgemm.cpp).
#
#   scripts/test_hw.sh 1 [--gpu] [--sizes "128 256 ..."] [--np "1 2 ..."]
#
# Builds the tool if it is missing, then runs every (n, np) pair with n divisible by np under a 30 s
# limit each and checks "Result verified" + the ANX_JSON record. Exit: 0 all passed, 1 a failure,
# 2 a timeout (and no failure) — the reference's convention, which run_hw.sh acts on.
set -u
ROOT=$(cd "$(dirname "$(realpath "$0")")/.." && pwd)
BIN="$ROOT/cuda-mpi-gpu-cluster-programming_amd/bin"
HW=${1:-}
shift || true
SIZES="128 256 512 1024 2048"
NPS="1 2 3 4 5 6 7 8"
GPU=""
while [ $# -gt 0 ]; do
  case $1 in
    --gpu) GPU="--gpu" ;;
    --sizes) SIZES=$2; shift ;;
    --np) NPS=$2; shift ;;
    *) echo "unknown option $1"; exit 1 ;;
  esac
  shift
done
if [ "$HW" != "1" ]; then
  echo "usage: $0 1 [--gpu] [--sizes LIST] [--np LIST]   (homework 1 = DGEMM is the only homework)"
  exit 1
fi
if [ ! -x "$BIN/anx_dgemm" ] || [ ! -x "$BIN/anxrun" ]; then
  echo "building anx_dgemm ..."
  cmake -S "$ROOT" -B "$ROOT/build" -G Ninja > /dev/null && cmake --build "$ROOT/build" --target anx_dgemm anxrun > /dev/null ||
    { echo "build failed"; exit 1; }
fi
fail=0
tmo=0
for n in $SIZES; do
  for np in $NPS; do
    if [ $((n % np)) -ne 0 ]; then
      echo "skip n=$n np=$np (n not divisible by np)"
      continue
    fi
    out=$(timeout -k 5 30s "$BIN/anxrun" -np "$np" --timeout 25 "$BIN/anx_dgemm" "$n" $GPU 2>&1)
    rc=$?
    if [ $rc -eq 124 ] || [ $rc -eq 137 ]; then
      echo "TIMEOUT n=$n np=$np"
      tmo=1
    elif [ $rc -ne 0 ] || ! grep -q "Result verified" <<< "$out" || ! grep -q '^ANX_JSON' <<< "$out"; then
      echo "FAIL n=$n np=$np (rc=$rc)"
      echo "$out" | tail -5
      fail=1
    else
      grep -m1 "^n=" <<< "$out"
    fi
  done
done
if [ $fail -ne 0 ]; then echo "--- homework $HW: FAILED ---"; exit 1; fi
if [ $tmo -ne 0 ]; then echo "--- homework $HW: INCONCLUSIVE (timeout) ---"; exit 2; fi
echo "--- homework $HW: PASSED ---"
