"""Scaffolder, static checks (K5) and the project collector (E3)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/llvm/bin/clang++"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="no ROCm clang")
def test_scaffold_op_compiles_for_gfx950(tmp_path):
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "scaffold.py"), "op", "my_scale", "--root",
                          str(tmp_path)], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stderr
    hip = tmp_path / "csrc" / "src" / "hip" / "my_scale.hip"
    capi = tmp_path / "csrc" / "src" / "my_scale_capi.cpp"
    assert hip.exists() and capi.exists() and (tmp_path / "tests" / "test_my_scale.py").exists()
    for src, lang in ((hip, "hip"), (capi, "c++")):
        r = subprocess.run([HIPCC, "-x", lang, "--offload-arch=gfx950", "-O2", "-std=c++17", "-c", str(src), "-o",
                            str(tmp_path / (src.name + ".o"))] if lang == "hip" else
                           [HIPCC, "-std=c++17", "-D__HIP_PLATFORM_AMD__", "-isystem", "/opt/rocm/include", "-c",
                            str(src), "-o", str(tmp_path / (src.name + ".o"))], capture_output=True, text=True,
                           timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
    again = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "scaffold.py"), "op", "my_scale", "--root",
                            str(tmp_path)], capture_output=True, text=True, timeout=60)
    assert again.returncode != 0 and "refusing to overwrite" in again.stderr


def test_scaffold_gpu_script(tmp_path):
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "scaffold.py"), "gpu-script", "probe", "--root",
                          str(tmp_path)], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stderr
    text = (tmp_path / "scripts" / "gpu_probe.sh").read_text()
    assert "timeout -k 10" in text and "&&" in text and "set -o pipefail" in text
    assert subprocess.run(["bash", "-n", str(tmp_path / "scripts" / "gpu_probe.sh")]).returncode == 0


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="no ROCm clang")
def test_lint_clean():
    r = subprocess.run(["bash", os.path.join(ROOT, "scripts", "lint.sh")], capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]


def test_collect_project(tmp_path):
    out = tmp_path / "project.txt"
    r = subprocess.run(["bash", os.path.join(ROOT, "scripts", "collect_project.sh"), str(out)], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    text = out.read_text()
    assert "===== csrc/src/hip/winograd.hip" in text and "===== bench.py" in text
