#!/bin/bash
# Multi-node orchestrator (the reference's scripts/2_final_multi_machine.sh):
# reachability, per-node inventory, code sync, per-node build, then every multi-rank version run
# ACROSS the nodes (one `anxrun --nnodes N --node-rank r` per node: the TCP host mesh / RCCL
# bootstrap spans them), parsed into the harness's 20-column CSV and a summary table.
#
# usage: scripts/run_cluster.sh --hostfile FILE [--versions "v2.1 v2.2 v4 v5"] [--batch N] [--iters K]
#            [--ppn N] [--port P] [--shared-fs] [--no-build] [--local] [--dry-run] [--out DIR]
#
# hostfile: one node per line, "[user@]host [ranks]" ('#' starts a comment). The first line is the
#   master: this machine, node rank 0, and the rendezvous address of every other node. ranks: ranks
#   on that node (default --ppn, else the node's GPU count for GPU versions and 1 for CPU ones).
# Phases (each logged to <session>/orchestration.log):
#   1 reach      ssh -o BatchMode=yes to every worker (no key generation: set up keys yourself)
#   2 inventory  gfx target, GPU count, ROCm version and CPUs of every node; GPU versions need every
#                node to report gfx950 (the only build target: no arch union as in the reference's
#                -gencode list)
#   3 sync       rsync of the tree minus .git / build / logs to the same path on every worker
#                (skipped with --shared-fs)
#   4 build      __graft_entry__ build on every node in parallel (skipped with --no-build)
#   5 run        per version: workers' anxrun in the background over ssh, the master's in the
#                foreground; the master's ANX_JSON is parsed; the checksum must equal the
#                single-process reference (V1 for CPU versions, V3 with direct convs for GPU ones)
# --local:   every host is this machine (no ssh / rsync; nodes are separate anxrun instances on
#            127.0.0.1) — how the CPU tests exercise the whole flow.
# --dry-run: print each phase's commands instead of running them.
set -uo pipefail
source "$(dirname "$0")/common.sh"

HOSTFILE=""; VERSIONS="v2.1 v2.2 v4 v5"; BATCH=2; ITERS=2; PPN=""; PORT=29650; SHARED=0; BUILD=1; LOCAL=0
DRY=0; LOGDIR="$ANX_ROOT/logs"; TMO=600
while [ $# -gt 0 ]; do
  case "$1" in
    --hostfile) HOSTFILE="$2"; shift 2 ;;
    --versions) VERSIONS="$2"; shift 2 ;;
    --batch) BATCH="$2"; shift 2 ;;
    --iters) ITERS="$2"; shift 2 ;;
    --ppn) PPN="$2"; shift 2 ;;
    --port) PORT="$2"; shift 2 ;;
    --shared-fs) SHARED=1; shift ;;
    --no-build) BUILD=0; shift ;;
    --local) LOCAL=1; shift ;;
    --dry-run) DRY=1; shift ;;
    --out) LOGDIR="$2"; shift 2 ;;
    --timeout) TMO="$2"; shift 2 ;;
    *) echo "usage: run_cluster.sh --hostfile FILE [--versions LIST] [--batch N] [--iters K] [--ppn N]"
       echo "                      [--port P] [--shared-fs] [--no-build] [--local] [--dry-run] [--out DIR]"
       exit 2 ;;
  esac
done
[ -n "$HOSTFILE" ] && [ -f "$HOSTFILE" ] || { echo "run_cluster: --hostfile FILE is required"; exit 2; }

HOSTS=(); RANKS=()
while read -r line; do
  line="${line%%#*}"
  read -r h r _ <<< "$line"
  [ -z "${h:-}" ] && continue
  if [ -n "${r:-}" ] && ! [[ "$r" =~ ^[0-9]+$ && "$r" -ge 1 ]]; then echo "run_cluster: bad ranks '$r' for $h"; exit 2; fi
  HOSTS+=("$h"); RANKS+=("${r:-}")
done < "$HOSTFILE"
NN=${#HOSTS[@]}
[ "$NN" -ge 1 ] || { echo "run_cluster: no hosts in $HOSTFILE"; exit 2; }
MASTER=${HOSTS[0]#*@}
[ "$LOCAL" -eq 1 ] && MASTER=127.0.0.1

TS=$(date +%Y%m%d_%H%M%S)
SESSION="cluster_${TS}_${NN}nodes"
OUT="$LOGDIR/$SESSION"
mkdir -p "$OUT"
OLOG="$OUT/orchestration.log"
CSV="$OUT/summary_report_${SESSION}.csv"
csv_init "$CSV"
GIT=$(git -C "$ANX_ROOT" rev-parse --short HEAD 2>/dev/null || echo unknown)
log() { echo "[$(date +%H:%M:%S)] $*" | tee -a "$OLOG"; }

# remote NODE_INDEX CMD: run CMD on that node (bash -c locally for the master and in --local mode)
remote() {
  local i="$1" cmd="$2"
  if [ "$DRY" -eq 1 ]; then
    if [ "$LOCAL" -eq 1 ] || [ "$i" -eq 0 ]; then echo "DRY local: $cmd"; else echo "DRY ssh ${HOSTS[$i]}: $cmd"; fi
    return 0
  fi
  if [ "$LOCAL" -eq 1 ] || [ "$i" -eq 0 ]; then bash -c "$cmd"; else
    ssh -o BatchMode=yes -o ConnectTimeout=10 "${HOSTS[$i]}" "$cmd"; fi
}

log "session $SESSION: $NN node(s), master $MASTER, versions: $VERSIONS, batch $BATCH"
# ---- 1 reach
for i in $(seq 1 $((NN - 1))); do
  if [ "$LOCAL" -eq 1 ]; then continue; fi
  if remote "$i" "true" >> "$OLOG" 2>&1; then log "reach ${HOSTS[$i]}: ok"; else
    log "reach ${HOSTS[$i]}: FAILED (ssh -o BatchMode=yes; install a key with ssh-copy-id first)"; exit 3; fi
done
# ---- 2 inventory
INV_CMD='a=$( (/opt/rocm/bin/rocm_agent_enumerator 2>/dev/null || true) | grep -v "^gfx000$" || true); \
g=$(printf "%s" "$a" | grep -c . || true); t=${a%%$'"'"'\n'"'"'*}; \
v=$(cat /opt/rocm/.info/version 2>/dev/null || echo none); echo "arch=${t:-none} gpus=$g rocm=$v cpus=$(nproc)"'
declare -a ARCH GPUS
ALL_GFX950=1
for i in $(seq 0 $((NN - 1))); do
  inv=$(remote "$i" "$INV_CMD" 2>> "$OLOG" | tail -1)
  [ "$DRY" -eq 1 ] && inv="arch=gfx950 gpus=${RANKS[$i]:-1} rocm=dry cpus=1"
  ARCH[$i]=$(sed -n 's/.*arch=\([^ ]*\).*/\1/p' <<< "$inv"); GPUS[$i]=$(sed -n 's/.*gpus=\([0-9]*\).*/\1/p' <<< "$inv")
  log "inventory ${HOSTS[$i]}: ${inv:-unreachable}"
  [ "${ARCH[$i]}" = gfx950 ] && [ "${GPUS[$i]:-0}" -ge 1 ] || ALL_GFX950=0
done
# ---- 3 sync
if [ "$LOCAL" -eq 0 ] && [ "$SHARED" -eq 0 ]; then
  for i in $(seq 1 $((NN - 1))); do
    cmd="rsync -az --delete --exclude .git/ --exclude build/ --exclude logs/ --exclude gpurun_out/ '$ANX_ROOT/' '${HOSTS[$i]}:$ANX_ROOT/'"
    if [ "$DRY" -eq 1 ]; then echo "DRY local: $cmd"; continue; fi
    remote "$i" "mkdir -p '$ANX_ROOT'" >> "$OLOG" 2>&1 && bash -c "$cmd" >> "$OLOG" 2>&1 || { log "sync ${HOSTS[$i]}: FAILED"; exit 3; }
    log "sync ${HOSTS[$i]}: ok"
  done
fi
# ---- 4 build (every node in parallel; in --local mode once)
BUILD_OK=1; BUILD_MSG=ok
if [ "$BUILD" -eq 1 ]; then
  pids=()
  for i in $(seq 0 $((NN - 1))); do
    [ "$LOCAL" -eq 1 ] && [ "$i" -gt 0 ] && break
    if [ "$DRY" -eq 1 ]; then remote "$i" "cd '$ANX_ROOT' && python3 __graft_entry__.py build"; continue; fi
    remote "$i" "cd '$ANX_ROOT' && python3 __graft_entry__.py build" > "$OUT/build_node$i.log" 2>&1 &
    pids+=($!)
  done
  for p in "${pids[@]}"; do wait "$p" || { BUILD_OK=0; BUILD_MSG=build_failed; }; done
  log "build: $BUILD_MSG"
fi

# ---- 5 run
declare -A REF_SUM=()
ranks_on() {  # node, version -> ranks on that node
  local i="$1" v="$2"
  if [ -n "${RANKS[$i]}" ]; then echo "${RANKS[$i]}"; elif [ -n "$PPN" ]; then echo "$PPN";
  elif [ "$v" = v4 ] || [ "$v" = v5 ]; then echo "${GPUS[$i]:-1}"; else echo 1; fi
}
gpu_args() { echo "--lrn-alpha-mode div_n --conv2-algo direct --conv1-algo direct --check"; }
reference() {  # version -> checksum of the single-process run on the master
  local dev="$1" log="$OUT/ref_$1.log" v=v1 extra=""
  [ "$dev" = gpu ] && { v=v3; extra=$(gpu_args); }
  [ -n "${REF_SUM[$dev]:-}" ] && return
  if [ "$DRY" -eq 1 ]; then echo "DRY local: anx --version $v"; REF_SUM[$dev]=dry; return; fi
  run_and_classify "$log" "$TMO" "$ANX_BIN/anx" --version "$v" --batch "$BATCH" --init rand --iters "$ITERS" $extra > /dev/null
  read -r _ _ _ sum _ < <(parse_anx_json "$log")
  REF_SUM[$dev]="$sum"
}
idx=0
for v in $VERSIONS; do
  idx=$((idx + 1))
  dev=cpu; extra=""
  case "$v" in v4|v5) dev=gpu; extra=$(gpu_args) ;; v2.1|v2.2) ;; *) log "skip $v: not a multi-rank version"; continue ;; esac
  if [ "$dev" = gpu ] && [ "$ALL_GFX950" -eq 0 ]; then
    log "skip $v: not every node reports a gfx950 GPU"
    summary_add "$v" "-" "$BATCH" NA NA "SKIP(no_gfx950)" NA NA
    continue
  fi
  reference "$dev"
  np=0
  for i in $(seq 0 $((NN - 1))); do np=$((np + $(ranks_on "$i" "$v"))); done
  port=$((PORT + idx))
  args="--version $v --batch $BATCH --init rand --iters $ITERS $extra"
  log "run $v: $np ranks over $NN node(s), rendezvous $MASTER:$port"
  pids=()
  for i in $(seq $((NN - 1)) -1 0); do
    n=$(ranks_on "$i" "$v")
    cmd="cd '$ANX_ROOT' && timeout -k 10 $TMO '$ANX_BIN/anxrun' -np $n --nnodes $NN --node-rank $i --master-addr $MASTER --port $port --timeout $((TMO - 30)) '$ANX_BIN/anx' $args"
    if [ "$i" -gt 0 ] && [ "$DRY" -eq 1 ]; then remote "$i" "$cmd"
    elif [ "$i" -gt 0 ]; then
      remote "$i" "$cmd" > "$OUT/run_${v}_node$i.log" 2>&1 &
      pids+=($!)
    fi
  done
  log0="$OUT/run_${v}_np${np}.log"
  if [ "$DRY" -eq 1 ]; then
    remote 0 "$cmd"; cls=0; t=NA; shape=13x13x256; first=NA; sum=dry; err=NA
  else
    cls=$(run_and_classify "$log0" "$((TMO + 30))" bash -c "$cmd")
    read -r t shape first sum err < <(parse_anx_json "$log0")
  fi
  for p in "${pids[@]}"; do wait "$p" || { [ "$cls" = 0 ] && cls=3; }; done
  status=OK; msg=ok; sym="✔"
  if [ "$DRY" -eq 1 ]; then status=DRY; msg=dry_run
  elif [ "$cls" != 0 ]; then status="FAIL($cls)"; msg="run_failed_class_$cls"; sym="✘"
  elif [ "$shape" != 13x13x256 ]; then status=BADSHAPE; msg="shape_$shape"; sym="✘"
  elif [ "$sum" != "${REF_SUM[$dev]}" ]; then status=MISMATCH; msg="checksum_differs"; sym="✘"
  elif [ "$dev" = gpu ] && { [ "$err" = NA ] || ! python3 -c "import sys; sys.exit(0 if float('$err') < 1e-3 else 1)"; }; then
    status=ORACLE; msg="max_abs_err_$err"; sym="✘"
  fi
  csv_row "$CSV" "$SESSION" "CLUSTER_${NN}nodes" "$GIT" "$(date +%s)" "$v" "$np" "$OUT/build_node0.log" "$BUILD_OK" \
    "$BUILD_MSG" "$log0" "$([ "$cls" = 0 ] && echo 1 || echo 0)" "" "$msg" "$([ "$t" != NA ] && echo 1 || echo 0)" "" \
    "$sym" "$status" "$t" "$shape" "$first"
  summary_add "$v" "$np" "$BATCH" "$t" "$shape" "$status" "$sum" "${err:-NA}"
done
summary_print | tee "$OUT/summary.txt"
log "csv: $CSV"
grep -q '✘' "$CSV" && exit 1
exit 0
