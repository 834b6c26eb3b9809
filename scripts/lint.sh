#!/bin/bash
# Static checks (no clang-tidy in this image): every C++/HIP source through the
# compiler with -Wall -Wextra -Wshadow as errors (syntax-only, host and gfx950 device passes), and
# every Python file byte-compiled.
set -uo pipefail
cd "$(dirname "$0")/.."
CXX=/opt/rocm/llvm/bin/clang++
flags=(-std=c++17 -Icsrc/include -isystem /opt/rocm/include -Wall -Wextra -Wshadow -Werror -Wno-unused-parameter -fsyntax-only)
fail=0
for f in $(git ls-files 'csrc/*.cpp' 'csrc/**/*.cpp'); do
  if grep -q -e '<<<' -e '\.hip"' "$f"; then  # HIP-language .cpp (CMake LANGUAGE HIP)
    $CXX -x hip --offload-arch=gfx950 "${flags[@]}" "$f" || { echo "LINT FAIL: $f"; fail=1; }
  else
    $CXX "${flags[@]}" -D__HIP_PLATFORM_AMD__ "$f" || { echo "LINT FAIL: $f"; fail=1; }
  fi
done
for f in $(git ls-files 'csrc/**/*.hip'); do
  $CXX -x hip --offload-arch=gfx950 "${flags[@]}" "$f" || { echo "LINT FAIL: $f"; fail=1; }
done
# Barrier discipline: every workgroup barrier in a kernel goes through anx::hip::lds_barrier<VM>()
# (anx/hip_sync.hpp: lgkmcnt(0) [+ vmcnt(VM)] before s_barrier). A bare s_barrier left this wave's LDS
# writes in flight past the barrier once (commit 52f2708).
bare=$(git grep -n '__builtin_amdgcn_s_barrier' -- 'csrc/*' ':!csrc/include/anx/hip_sync.hpp' | grep -v '^[^:]*:[0-9]*: *//')
if [ -n "$bare" ]; then echo "LINT FAIL: bare s_barrier (use anx::hip::lds_barrier):"; echo "$bare"; fail=1; fi
python3 -m compileall -q cuda-mpi-gpu-cluster-programming_amd tools tests bench.py __graft_entry__.py anx.py \
  > /dev/null || fail=1
[ $fail -eq 0 ] && echo "lint: OK"
exit $fail
