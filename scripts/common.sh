#!/bin/bash
# Shared helpers of the run harness (the reference's scripts/common_test_utils.sh):
# GPU detection, CSV logging in the reference's 20-column schema, a command runner with a failure
# taxonomy, output parsing and an ASCII summary table. Unlike the reference harness, a wrong output
# shape or a checksum mismatch is a FAILURE, not "OK".

ANX_ROOT="${ANX_ROOT:-$(cd "$(dirname "${BASH_SOURCE[0]}")/.." && pwd)}"
ANX_BIN="$ANX_ROOT/cuda-mpi-gpu-cluster-programming_amd/bin"
CSV_HEADER="SessionID,MachineID,GitCommit,EntryTimestamp,ProjectVariant,NumProcesses,MakeLogFile,BuildSucceeded,BuildMessage,RunLogFile,RunCommandSucceeded,RunEnvironmentWarning,RunMessage,ParseSucceeded,ParseMessage,OverallStatusSymbol,OverallStatusMessage,ExecutionTime_ms,OutputShape,OutputFirst5Values"
declare -a SUMMARY_ROWS=()

# gfx target of the first GPU (the reference probed nvidia-smi compute_cap with sm_50/sm_75 guesses;
# here there is exactly one target, gfx950, and its absence is reported, never guessed).
detect_gpu_arch() {
  if command -v rocminfo >/dev/null 2>&1; then
    # no `grep -m1`: an early grep exit SIGPIPEs rocminfo and, under pipefail, also printed "none"
    local a
    a=$(rocminfo 2>/dev/null | grep -o 'gfx[0-9a-f]*' || true)
    a=${a%%$'\n'*}
    echo "${a:-none}"
  else
    echo "none"
  fi
}

gpu_count() {
  python3 -c "import torch; print(torch.cuda.device_count())" 2>/dev/null || echo 0
}

csv_init() {  # $1 = csv path
  [ -f "$1" ] || echo "$CSV_HEADER" > "$1"
}

csv_row() {  # csv path, then the 20 fields
  local f="$1"; shift
  local IFS=,
  echo "$*" >> "$f"
}

# Run a command with a log; classify failures like the reference (env/device 2, comm config 3,
# segfault 4, other 1) and echo the class.
run_and_classify() {  # logfile, timeout_s, cmd...
  local log="$1" tmo="$2"; shift 2
  timeout -k 10 "$tmo" "$@" > "$log" 2>&1
  local rc=$?
  if [ $rc -eq 0 ]; then echo 0; return; fi
  if [ $rc -eq 124 ] || [ $rc -eq 137 ]; then echo 5; return; fi           # watchdog timeout
  if grep -qiE 'no GPU|needs a GPU|hipError|HIP .*error|invalid device' "$log"; then echo 2; return; fi
  if grep -qiE 'HostComm|RCCL|connect timeout|bad rank' "$log"; then echo 3; return; fi
  if [ $rc -eq 139 ] || grep -qi 'segmentation fault' "$log"; then echo 4; return; fi
  echo 1
}

# Parse an ANX_JSON record: prints "time_ms shape first5 checksum max_abs_err" (time = warm if
# present; max_abs_err vs the fp64 oracle when the run had --check, else NA).
parse_anx_json() {  # logfile
  python3 - "$1" <<'EOF'
import json, sys
rec = None
for line in open(sys.argv[1], errors="replace"):
    if line.startswith("ANX_JSON "):
        rec = json.loads(line[9:])
if rec is None:
    print("NA NA NA NA NA"); sys.exit(0)
t = rec.get("warm_ms") or rec.get("cold_ms")
first = rec.get("first10") or []
print(f"{t:.4f} {'x'.join(map(str, rec['shape']))} {'|'.join(str(v) for v in first[:5]) or 'NA'} {rec['checksum']} {rec.get('max_abs_err') if rec.get('max_abs_err') is not None else 'NA'}")
EOF
}

summary_add() { SUMMARY_ROWS+=("$*"); }

summary_print() {
  printf '%-8s %-4s %-6s %-12s %-12s %-10s %-11s %s\n' VERSION NP BATCH TIME_MS SHAPE STATUS CHECKSUM MAX_ABS_ERR
  printf '%s\n' "-------------------------------------------------------------------------------"
  for r in "${SUMMARY_ROWS[@]}"; do
    # shellcheck disable=SC2086
    printf '%-8s %-4s %-6s %-12s %-12s %-10s %-11s %s\n' $r
  done
}
