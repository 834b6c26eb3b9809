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
python3 -m compileall -q cuda-mpi-gpu-cluster-programming_amd tools tests bench.py __graft_entry__.py anx.py \
  > /dev/null || fail=1
[ $fail -eq 0 ] && echo "lint: OK"
exit $fail
