#!/bin/bash
# One parameterised runner for every GPU session (run on the box through gpurun):
#
#   bash scripts/gpu.sh SESSION [SESSION ...]
#
# Sessions (each GPU step has its own time limit; the chain stops at the first failure, so a fault,
# abort or timeout ends the call):
#   tests    all GPU tests (one pytest process)          smoke   __graft_entry__ smoke()
#   bench    bench.py defaults                           sweep   tools/sweep_batch.py 64..600 images
#   ab       tools/ab_variants.py with $AB_ARMS (and $AB_BATCH, $AB_LANES)
#   prof     rocprofv3 kernel trace of the bench step    pmc     PMC passes (SQ x2, TCC x2) of the bench step
#   full     bf16 full-AlexNet bench + kernel trace     matrix  scripts/run_matrix.sh at batch 1 and 256
#   peak     sustained f32 MFMA peak (anx_mfmapeak)     workloads  bench.py --workload v4 / v5 at N=1
#   versions native V3/V4/V5 CLI (shared-GPU ranks)    markers rocprofv3 marker trace of a V5 peer run
# Outputs land in gpurun_out/ (merged back by gpurun).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B=cuda-mpi-gpu-cluster-programming_amd/bin
O=gpurun_out
BARGS=${BENCH_ARGS:-}

run() {  # run NAME SECONDS CMD...: one GPU step with its own limit and log
  local name=$1 secs=$2
  shift 2
  echo "== $name: $*"
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  tail -3 "$O/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "== $name FAILED rc=$rc"; exit $rc; fi
}
pmc() {  # pmc NAME COUNTERS...: one counter pass over a short bench run
  local name=$1
  shift
  echo "== pmc $name: $*"
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$O/$name" -o pmc -- \
    python3 bench.py --steps 3 --warmup 1 $BARGS > "$O/$name.log" 2>&1 || { echo "== pmc $name FAILED"; exit 1; }
}

for s in "$@"; do
  case $s in
    tests) run tests 900 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread ;;
    smoke) run smoke 300 python __graft_entry__.py smoke ;;
    bench) run bench 300 python bench.py --steps 20 --warmup 5 $BARGS ;;
    sweep) run sweep 600 python tools/sweep_batch.py --batches ${SWEEP:-64,128,256,300,600} --rounds 3 --iters 10 ;;
    ab) run ab 900 python tools/ab_variants.py --arms "${AB_ARMS:-|conv1_occ=3}" --batch "${AB_BATCH:-300}" \
          --lanes "${AB_LANES:-1}" --rounds "${AB_ROUNDS:-5}" ;;
    prof) run prof 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run -- python3 bench.py --steps 10 --warmup 3 $BARGS ;;
    pmc)
      pmc pmc1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE SQ_INSTS_MFMA
      pmc pmc2 SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INST_LEVEL_VMEM
      pmc pmc3 TCC_HIT_sum TCC_MISS_sum
      pmc pmc4 FETCH_SIZE
      pmc pmc5 WRITE_SIZE ;;
    full)
      run full_bench 300 python bench.py --model full --steps 20 --warmup 5
      run full_prof 300 rocprofv3 --kernel-trace --stats -d "$O/full_prof" -o run -- python3 bench.py --model full --steps 10 --warmup 3 ;;
    matrix)
      run matrix_b1 400 bash scripts/run_matrix.sh --no-build --batch 1 --iters 3 --out "$O/matrix"
      run matrix_b256 600 bash scripts/run_matrix.sh --no-build --batch 256 --iters 1 --out "$O/matrix" ;;
    peak) run peak 120 bash -c "$B/anx_mfmapeak --waves 1 && $B/anx_mfmapeak --waves 2 && $B/anx_mfmapeak --waves 4" ;;
    workloads)
      run wl_v4 300 python bench.py --workload v4 --steps 10 --warmup 3
      run wl_v5 300 python bench.py --workload v5 --steps 10 --warmup 3 ;;
    versions)
      run v3_b1 120 $B/anx --version v3 --iters 20 --check
      run v4_np2 180 $B/anxrun -np 2 --timeout 150 -- $B/anx --version v4 --batch 8 --iters 5 --check
      run v5_np4 180 $B/anxrun -np 4 --timeout 150 -- $B/anx --version v5 --transport peer --batch 8 --iters 5 --check ;;
    # the profiler wraps each rank (anxrun only forks; it never touches the GPU)
    markers) run markers 300 $B/anxrun -np 2 --timeout 240 -- rocprofv3 --marker-trace --kernel-trace --stats \
               -d "$O/markers" -o "rank_%pid%" -- $B/anx --version v5 --transport peer --batch 32 --iters 10 ;;
    *) echo "unknown session $s"; exit 2 ;;
  esac
done
