"""Every staged version end to end on CPU ranks (gloo), through the same launcher a user runs
(``python -m anx launch --np N -- --version ...``). Multi-rank outputs must equal the serial V1
output exactly — shape 13x13x256 and every value (the reference's V2.2/V4 at np>=2 failed this)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_cli(args, np_=None, timeout=600):
    base = [sys.executable, "-c", "import anx.__main__ as m; m.main()"]
    cmd = base + (["launch", "--np", str(np_), "--timeout", str(timeout), "--"] if np_ else ["run"]) + args
    env = dict(os.environ, OMP_NUM_THREADS="1", PYTHONPATH=ROOT)
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout + 60, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-4000:]
    recs = [json.loads(l[len("ANX_JSON "):]) for l in out.stdout.splitlines() if l.startswith("ANX_JSON ")]
    assert len(recs) == 1, out.stdout
    return recs[0], out.stdout


@pytest.fixture(scope="module")
def serial():
    rec, _ = run_cli(["--version", "v1", "--init", "rand", "--seed", "3", "--batch", "2"])
    return rec


def test_v1_contract_lines():
    rec, out = run_cli(["--version", "v1"])
    assert "AlexNet Serial Forward Pass completed in" in out
    assert rec["shape"] == [13, 13, 256]
    assert rec["first10"][:3] == pytest.approx([44.4152, 42.4612, 40.6967], abs=2e-4)


@pytest.mark.parametrize("np_", [2, 3])
def test_v21_broadcast_all(serial, np_):
    rec, out = run_cli(["--version", "v2.1", "--init", "rand", "--seed", "3", "--batch", "2"], np_)
    assert "Execution Time:" in out and rec["np"] == np_
    assert rec["checksum"] == serial["checksum"]


@pytest.mark.parametrize("np_", [2, 4, 5])
def test_v22_scatter_halo(serial, np_):
    rec, out = run_cli(["--version", "v2.2", "--init", "rand", "--seed", "3", "--batch", "2"], np_)
    assert "shape: 13x13x256" in out
    assert rec["checksum"] == serial["checksum"]


@pytest.mark.parametrize("version,extra", [
    ("v4", []), ("v4", ["--decomp", "per_layer"]), ("v5", []), ("v5", ["--strategy", "batch"]),
])
def test_gpu_versions_cpu_rehearsal(serial, version, extra):
    rec, out = run_cli(["--version", version, "--cpu-rehearsal", "--lrn-alpha-mode", "div_n", "--init", "rand",
                        "--seed", "3", "--batch", "2", *extra], 3)
    assert "Final Output Shape: 13x13x256" in out
    assert rec["checksum"] == serial["checksum"]


@pytest.mark.parametrize("np_", [2, 4])
def test_v22_filter_parallel(serial, np_):
    """P7: Conv2 filters split over CPU ranks with an LRN channel halo == the serial V1 output."""
    rec, _ = run_cli(["--version", "v2.2", "--strategy", "filter", "--init", "rand", "--seed", "3", "--batch", "2"],
                     np_)
    assert rec["shape"] == [13, 13, 256]
    assert rec["checksum"] == serial["checksum"]
