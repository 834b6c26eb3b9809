set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local n=$1 s=$2; shift 2; echo "== $n"; timeout -k 10 $s "$@" > gpurun_out/$n.log 2>&1; local rc=$?; tail -3 gpurun_out/$n.log | cut -c1-300; [ $rc -eq 0 ] || { echo "== $n FAILED rc=$rc"; exit $rc; }; }
run tests 600 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread
run bench 200 python bench.py --steps 20 --warmup 5
run ab 600 python tools/ab_variants.py --arms "|conv1_occ=3|conv1_occ=2|conv2_occ=1|conv1_occ=3;conv2_occ=1" --batch 128 --lanes 2 --rounds 5
