#!/bin/bash
# Concatenate the project's sources and docs into one text file for review (the
# reference's collect_project.sh / collect_p_docs.sh). usage: scripts/collect_project.sh [OUT]
set -euo pipefail
cd "$(dirname "$0")/.."
out="${1:-project.txt}"
{
  echo "# anx project dump — $(git rev-parse --short HEAD 2>/dev/null || echo nogit) — $(date -u +%F)"
  git ls-files 'README.md' 'docs/*.md' 'CMakeLists.txt' 'csrc/**' 'cuda-mpi-gpu-cluster-programming_amd/**/*.py' \
    '*.py' 'tools/*.py' 'scripts/*.sh' 'tests/*.py' | while read -r f; do
    echo
    echo "===== $f ($(wc -l < "$f") lines) ====="
    cat "$f"
  done
} > "$out"
echo "wrote $out ($(wc -l < "$out") lines)"
