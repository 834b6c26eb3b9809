"""Host AddressSanitizer run of the native runtime (the reference only recommends
valgrind / cuda-memcheck, final_project/PROBLEMS.txt:86-93).

Builds the CMake project with -DANX_HOST_ASAN=ON into build/asan_out (never over the in-tree
library; device code is not sanitized — GPU sanitizers are not available on this pool) and runs the
multi-rank host paths clean: V1, V2.2 scatter + halo exchange over the TCP host comm at 2-4 ranks
(the same host staging / planner / transfer code V4 runs around its GPU tile), the exact planner for
np 1..8, and the V5 transfer schedule (record-only transports) at 2-4 ranks. Any ASan report or
leak fails the run.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "build", "asan")
OUT = os.path.join(ROOT, "build", "asan_out")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:exitcode=23", OMP_NUM_THREADS="1")

pytestmark = pytest.mark.skipif(shutil.which("cmake") is None, reason="cmake missing")


@pytest.fixture(scope="module")
def asan_bin():
    cxx = "/opt/rocm/llvm/bin/clang++"
    if not os.path.exists(cxx):
        pytest.skip("ROCm clang missing")
    gen = ["-G", "Ninja"] if shutil.which("ninja") else []
    subprocess.run(["cmake", "-S", ROOT, "-B", BUILD, *gen, f"-DCMAKE_CXX_COMPILER={cxx}",
                    "-DCMAKE_HIP_ARCHITECTURES=gfx950", "-DCMAKE_BUILD_TYPE=Release", "-DANX_HOST_ASAN=ON",
                    f"-DANX_OUTPUT_ROOT={OUT}"], check=True, capture_output=True, timeout=300)
    r = subprocess.run(["cmake", "--build", BUILD, "-j", str(min(8, os.cpu_count() or 4)), "--target", "anx_cli",
                        "anxrun"], capture_output=True, text=True, timeout=1800)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return os.path.join(OUT, "bin")


def run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=ENV)
    text = r.stdout + r.stderr
    assert "AddressSanitizer" not in text and "LeakSanitizer" not in text, text[-4000:]
    assert r.returncode == 0, text[-3000:]
    return r.stdout


def test_asan_v1(asan_bin):
    out = run([os.path.join(asan_bin, "anx"), "--version", "v1", "--check"])
    assert "44.4152 42.4612 40.6967" in out


@pytest.mark.parametrize("np_,decomp", [(2, "overlap"), (4, "overlap"), (3, "per_layer")])
def test_asan_v22_multirank(asan_bin, np_, decomp):
    b = asan_bin
    out = run([os.path.join(b, "anxrun"), "-np", str(np_), "--timeout", "200", os.path.join(b, "anx"), "--version",
               "v2.2", "--init", "rand", "--batch", "2", "--iters", "1", "--check", "--decomp", decomp])
    assert '"max_abs_err": 0.000000' in out or '"max_abs_err": 0.0' in out


@pytest.mark.parametrize("np_,split", [(2, "rows"), (3, "rows"), (4, "hybrid")])
def test_asan_v5_schedule(asan_bin, np_, split):
    b = asan_bin
    out = run([os.path.join(b, "anxrun"), "-np", str(np_), "--timeout", "120", os.path.join(b, "anx"), "--version",
               "v5", "--dry-run", "--split", split, "--batch", "3"])
    assert out.count("ANX_SCHEDULE") > 0
