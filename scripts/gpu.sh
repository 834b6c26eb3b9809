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
#   benchab  bench.py arms alternated $BENCH_REPS times: BENCH_AB="conv1_band=1|conv1_band=2" (';' joins
#            knobs of one arm), one JSON line per run into benchab.jsonl ($BENCH_STEPS timed steps)
#   bytes    per-kernel HBM bytes, clock and MFMA busy of the bench step (FETCH / WRITE passes)
#   wgemm    anx_wgemm Winograd GEMM A/B at 300 and 64 images; wgpmc: its clock / MFMA busy pass
#   halo     V5 halo pipeline A/B on shared-GPU peer ranks, 2-way rows: np {2,4} x chunks {1, auto}
#   tests_k  a subset of GPU tests: pytest -k "$TESTS_K" (one process)
#   ingest   tools/probe_ingest.py: the bench step with a concurrent 155 MB/step receive-side copy
#   libab    bench.py with the in-tree libanx vs an alternative build ($LIBAB/lib, e.g. ab_slp/: another
#            CMake configuration of the same sources), alternated $BENCH_REPS times into libab.jsonl
# Outputs land in gpurun_out/ (merged back by gpurun). This one script replaces the per-session
# wrappers of rounds 1-3.
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
    python3 bench.py --steps 3 --warmup 1 --no-full $BARGS > "$O/$name.log" 2>&1 || { echo "== pmc $name FAILED"; exit 1; }
}

for s in "$@"; do
  case $s in
    tests) run tests 900 python -u -m pytest tests -x -v -m gpu --timeout 170 --timeout-method thread ;;
    smoke) run smoke 300 python __graft_entry__.py smoke ;;
    bench) run bench 300 python bench.py --steps 20 --warmup 5 $BARGS ;;
    sweep) run sweep 600 python tools/sweep_batch.py --batches ${SWEEP:-64,128,256,300,600} --rounds 3 --iters 10 \
             ${SWEEP_ARGS:-} ;;
    ab) run ab 900 python tools/ab_variants.py --arms "${AB_ARMS:-|conv1_occ=3}" --batch "${AB_BATCH:-300}" \
          --lanes "${AB_LANES:-1}" --rounds "${AB_ROUNDS:-5}" ;;
    prof) run prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 bench.py --steps 10 --warmup 3 --no-full $BARGS ;;
    pmc)
      pmc pmc1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE SQ_INSTS_MFMA
      pmc pmc2 SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INST_LEVEL_VMEM
      pmc pmc3 TCC_HIT_sum TCC_MISS_sum
      pmc pmc4 FETCH_SIZE
      pmc pmc5 WRITE_SIZE ;;
    full)
      run full_bench 300 python bench.py --model full --steps 20 --warmup 5 $BARGS
      run full_prof 300 rocprofv3 --kernel-trace --stats -d "$O/full_prof" -o run -- python3 bench.py --model full --steps 10 --warmup 3 $BARGS ;;
    matrix)
      run matrix_b1 400 bash scripts/run_matrix.sh --no-build --batch 1 --iters 3 --out "$O/matrix"
      run matrix_b256 600 bash scripts/run_matrix.sh --no-build --batch 256 --iters 1 --out "$O/matrix" ;;
    peak) run peak 120 bash -c "$B/anx_mfmapeak --waves 1 && $B/anx_mfmapeak --waves 2 && $B/anx_mfmapeak --waves 4" ;;
    workloads)
      run wl_v4 300 python bench.py --workload v4 --steps 10 --warmup 3
      run wl_v5 300 python bench.py --workload v5 --steps 10 --warmup 3
      run wl_v5_root 300 python bench.py --workload v5 --input-source root --steps 10 --warmup 3 --no-b1 ;;
    ingest) run probe_ingest 600 python tools/probe_ingest.py ${INGEST_ARGS:-} ;;
    versions)
      run v3_b1 120 $B/anx --version v3 --iters 20 --check
      run v4_np2 180 $B/anxrun -np 2 --timeout 150 -- $B/anx --version v4 --batch 8 --iters 5 --check
      run v5_np4 180 $B/anxrun -np 4 --timeout 150 -- $B/anx --version v5 --transport peer --batch 8 --iters 5 --check ;;
    # the profiler wraps each rank (anxrun only forks; it never touches the GPU)
    markers) run markers 300 $B/anxrun -np 2 --timeout 240 -- rocprofv3 --marker-trace --kernel-trace --stats \
               -d "$O/markers" -o "rank_%pid%" -- $B/anx --version v5 --transport peer --batch 32 --iters 10 ;;
    tests_k) run tests_k 900 python -u -m pytest tests -x -v -m gpu -k "${TESTS_K:?}" --timeout 240 --timeout-method thread ;;
    benchab)
      IFS='|' read -r -a arms <<< "${BENCH_AB:?BENCH_AB=arm|arm}"
      for rep in $(seq "${BENCH_REPS:-3}"); do
        for arm in "${arms[@]}"; do
          kargs=()
          IFS=';' read -r -a kvs <<< "$arm"
          for kv in "${kvs[@]}"; do  # k=v: an engine knob; --flag=v: a bench.py argument
            if [[ $kv == --* ]]; then kargs+=("$kv"); elif [ -n "$kv" ]; then kargs+=(--knob "$kv"); fi
          done
          echo "== benchab rep $rep arm '$arm'"
          timeout -k 10 200 python -u bench.py --steps "${BENCH_STEPS:-20}" --warmup 5 --no-b1 --no-full $BARGS "${kargs[@]}" \
            >> "$O/benchab.jsonl" 2>> "$O/benchab.err" || { echo "== benchab FAILED"; exit 1; }
          tail -1 "$O/benchab.jsonl" | cut -c1-160
        done
      done ;;
    libab)
      for rep in $(seq "${BENCH_REPS:-3}"); do
        for arm in intree "${LIBAB:?LIBAB=dir}"; do
          echo "== libab rep $rep arm $arm"
          if [ "$arm" = intree ]; then
            timeout -k 10 200 python -u bench.py --steps "${BENCH_STEPS:-20}" --warmup 5 --no-b1 --no-full $BARGS \
              >> "$O/libab_intree.jsonl" 2>> "$O/libab.err" || { echo "== libab FAILED"; exit 1; }
            tail -1 "$O/libab_intree.jsonl" | cut -c1-160
          else
            ANX_LIB="$arm/lib/libanx.so" timeout -k 10 200 python -u bench.py --steps "${BENCH_STEPS:-20}" --warmup 5 \
              --no-b1 --no-full $BARGS >> "$O/libab_alt.jsonl" 2>> "$O/libab.err" || { echo "== libab FAILED"; exit 1; }
            tail -1 "$O/libab_alt.jsonl" | cut -c1-160
          fi
        done
      done ;;
    c1abl)  # conv1_fused cost probes (build_abl: cmake -DANX_CONV1_ABL=ON -DANX_OUTPUT_ROOT=ab_abl), one lane
      for abl in ${C1ABL:-0 1 2 4 8 16 24 32 7 63}; do
        echo "== c1abl $abl"
        ANX_LIB=ab_abl/lib/libanx.so ANX_CONV1_ABL=$abl timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv \
          -d "$O/c1abl_$abl" -o run -- python3 bench.py --lanes 1 --steps 8 --warmup 2 --no-b1 --no-full --prewarm-s 0.5 \
          > "$O/c1abl_$abl.log" 2>&1 || { echo "== c1abl FAILED"; exit 1; }
        python3 tools/rocprof_summary.py "$(ls "$O"/c1abl_$abl/*kernel_trace.csv | head -1)" | grep -E "conv1_fused|gemm_kernel" \
          | cut -c1-200 | tee -a "$O/c1abl.md"
      done ;;
    bytes)
      BYARGS="--lanes 1 --steps 6 --warmup 2 --no-b1 --no-full --prewarm-s 0 $BARGS"
      timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace \
        --output-format csv -d "$O/pmc_fetch" -o run -- python3 bench.py $BYARGS > "$O/pmc_fetch.log" 2>&1 &&
      timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --kernel-trace \
        --output-format csv -d "$O/pmc_write" -o run -- python3 bench.py $BYARGS > "$O/pmc_write.log" 2>&1 &&
      python3 tools/pmc_clock.py "$O/pmc_fetch" "$O/pmc_write" > "$O/pmc_bytes.md" || { echo "== bytes FAILED"; exit 1; }
      cat "$O/pmc_bytes.md" ;;
    wgemm)
      run wg300 120 $B/anx_wgemm --images 300 --iters 20
      run wg64 120 $B/anx_wgemm --images 64 --iters 20 ;;
    wg45)  # Conv2 F(4x4,5x5) GEMM configurations vs the F(3x3,5x5) production GEMM (anx_wgemm --conv 4)
      run wg45_128 120 $B/anx_wgemm --conv 4 --images 128 --iters 20
      run wg45_300 120 $B/anx_wgemm --conv 4 --images 300 --iters 20 ;;
    wg45pmc)
      timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
        --kernel-trace --output-format csv -d "$O/wg45pmc" -o run -- $B/anx_wgemm --conv 4 --images 128 --iters 3 \
        > "$O/wg45pmc.log" 2>&1 && python3 tools/pmc_clock.py "$O/wg45pmc" | tee "$O/wg45pmc.md" || { echo "== wg45pmc FAILED"; exit 1; } ;;
    wgpmc)
      timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
        --kernel-trace --output-format csv -d "$O/wgpmc" -o run -- $B/anx_wgemm --images 300 --iters 3 \
        > "$O/wgpmc.log" 2>&1 && python3 tools/pmc_clock.py "$O/wgpmc" || { echo "== wgpmc FAILED"; exit 1; } ;;
    halo)  # the BASELINE V5 share: 256 images per 2-way row group (np 2: 256 images, np 4: 512)
      for np in 2 4; do
        for ch in 1 0; do
          run "halo_np${np}_c${ch}" 240 $B/anxrun -np $np --timeout 200 -- $B/anx --version v5 --transport peer \
            --batch $((np * ${HALO_SHARE:-128})) --row-ways 2 --iters 30 --init rand --chunks $ch
        done
      done ;;
    *) echo "unknown session $s"; exit 2 ;;
  esac
done
