#!/bin/bash
# Package a homework for submission (the reference's scripts/package_hw.sh):
#
#   scripts/package_hw.sh 1 <lastname> <firstname>   ->  hw1-<lastname>-<firstname>.tgz
#
# The archive is self-contained: the DGEMM source, the headers it includes (the host comm layer and
# the anxrun launcher it runs under) and a Makefile that builds both with hipcc for gfx950 — no
# CMake, no Python. The staged tree is built once before archiving, so a package that does not
# compile is never produced.
set -u
ROOT=$(cd "$(dirname "$(realpath "$0")")/.." && pwd)
if [ "$#" -ne 3 ]; then
  echo "usage: $0 <homework_number> <lastname> <firstname>   (example: $0 1 doe jane)"
  exit 1
fi
HW=$1
LAST=$(tr '[:upper:]' '[:lower:]' <<< "$2")
FIRST=$(tr '[:upper:]' '[:lower:]' <<< "$3")
if [ "$HW" != "1" ]; then echo "homework $HW does not exist (1 = DGEMM)"; exit 1; fi
NAME="hw${HW}-${LAST}-${FIRST}"
OUT="$PWD/$NAME.tgz"
STAGE=$(mktemp -d)
trap 'rm -rf "$STAGE"' EXIT
D="$STAGE/$NAME"
mkdir -p "$D/src" "$D/include/anx"
cp "$ROOT/csrc/src/versions/dgemm.cpp" "$ROOT/csrc/src/comm/host_comm.cpp" "$ROOT/csrc/src/runtime/launcher.cpp" "$D/src/"
cp "$ROOT/csrc/include/anx/comm.hpp" "$D/include/anx/"
for h in $(grep -ho '#include "anx/[a-z_]*\.hpp"' "$D/src/"*.cpp "$D/include/anx/comm.hpp" | sort -u | sed 's/.*"anx\/\(.*\)"/\1/'); do
  [ -f "$D/include/anx/$h" ] || cp "$ROOT/csrc/include/anx/$h" "$D/include/anx/"
done
cat > "$D/Makefile" <<'EOF'
# Homework 1: row-distributed fp64 DGEMM (host ranks over TCP, optional fp64 MFMA per rank on gfx950)
HIPCC ?= /opt/rocm/bin/hipcc
CXXFLAGS ?= -O2 -std=c++17 -Iinclude
all: template anxrun
template: src/dgemm.cpp src/host_comm.cpp
	$(HIPCC) --offload-arch=gfx950 $(CXXFLAGS) -o $@ $^
anxrun: src/launcher.cpp
	$(HIPCC) $(CXXFLAGS) -o $@ $^
clean:
	rm -f template anxrun
.PHONY: all clean
EOF
cat > "$D/README" <<EOF
Homework $HW (row-distributed DGEMM) — $FIRST $LAST
build: make            run: ./anxrun -np 4 ./template 1024 [--gpu]
EOF
echo "--- packaging homework $HW for $FIRST $LAST -> $OUT ---"
( cd "$D" && make -s > "$STAGE/build.log" 2>&1 ) || { echo "staged tree does not build:"; tail -20 "$STAGE/build.log"; exit 1; }
( cd "$D" && make -s clean )
tar czf "$OUT" -C "$STAGE" "$NAME" || { echo "tar failed"; exit 1; }
echo "--- homework $HW packaging: SUCCESS ($(tar tzf "$OUT" | wc -l) entries) ---"
