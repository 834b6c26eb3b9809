"""Homework side-track workflow (the reference's scripts/test_hw.sh, package_hw.sh,
run_hw.sh): test homework 1 (row-distributed DGEMM) over anxrun ranks, then package a
self-contained source tree that builds with a plain Makefile."""
import os
import shutil
import subprocess
import tarfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "cuda-mpi-gpu-cluster-programming_amd", "bin")

pytestmark = pytest.mark.skipif(not os.path.exists(os.path.join(BIN, "anx_dgemm")) or shutil.which("hipcc") is None
                                and not os.path.exists("/opt/rocm/bin/hipcc"), reason="tools / hipcc missing")


def sh(args, cwd, timeout=600):
    return subprocess.run(["bash", *args], cwd=cwd, capture_output=True, text=True, timeout=timeout,
                          env=dict(os.environ, OMP_NUM_THREADS="1"))


def test_run_hw_tests_then_packages(tmp_path):
    r = sh([os.path.join(ROOT, "scripts", "run_hw.sh"), "1", "Doe", "Jane", "--sizes", "128 256", "--np", "1 2 4"],
           tmp_path)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert r.stdout.count("Result verified") == 6 and "PASSED" in r.stdout
    tgz = tmp_path / "hw1-doe-jane.tgz"
    with tarfile.open(tgz) as t:
        names = set(t.getnames())
    assert {"hw1-doe-jane/Makefile", "hw1-doe-jane/src/dgemm.cpp", "hw1-doe-jane/include/anx/comm.hpp"} <= names


def test_test_hw_rejects_unknown_homework(tmp_path):
    r = sh([os.path.join(ROOT, "scripts", "test_hw.sh"), "7"], tmp_path, 60)
    assert r.returncode == 1 and "usage" in r.stdout


def test_test_hw_reports_skips_for_indivisible_rank_counts(tmp_path):
    r = sh([os.path.join(ROOT, "scripts", "test_hw.sh"), "1", "--sizes", "128", "--np", "3"], tmp_path, 120)
    assert r.returncode == 0 and "skip n=128 np=3" in r.stdout
