"""Native side tools: HW1 DGEMM (the reference's homework sweep, scripts/test_hw.sh: np x n with
n % np == 0, 30 s timeout), the conv micro-benchmark and the device-binding report."""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "cuda-mpi-gpu-cluster-programming_amd", "bin")
pytestmark = pytest.mark.skipif(not os.path.exists(os.path.join(BIN, "anx_dgemm")), reason="tools not built")


def run(cmd, timeout=60):
    return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout,
                          env=dict(os.environ, OMP_NUM_THREADS="1"))


@pytest.mark.parametrize("np_", [1, 2, 4])
@pytest.mark.parametrize("n", [128, 256])
def test_dgemm_sweep(np_, n):
    out = run([os.path.join(BIN, "anxrun"), "-np", str(np_), "--timeout", "30", os.path.join(BIN, "anx_dgemm"), str(n)])
    assert out.returncode == 0, out.stderr
    rec = json.loads(next(l for l in out.stdout.splitlines() if l.startswith("ANX_JSON"))[9:])
    assert rec["ok"] and rec["np"] == np_ and rec["n"] == n
    assert "Result verified" in out.stdout


@pytest.mark.parametrize("args", [["96"], ["256"]])
def test_dgemm_rejects_bad_sizes(args):
    """n not a power of two, or not divisible by np (3): fail-stop like MPI_Abort."""
    out = run([os.path.join(BIN, "anxrun"), "-np", "3", "--timeout", "30", os.path.join(BIN, "anx_dgemm"), *args])
    assert out.returncode != 0


def test_devinfo_ranks():
    out = run([os.path.join(BIN, "anxrun"), "-np", "3", os.path.join(BIN, "anx_devinfo")])
    assert out.returncode == 0
    assert [l.split()[1] for l in out.stdout.splitlines()] == ["0/3", "1/3", "2/3"]


@pytest.mark.gpu
def test_dgemm_gpu_mfma_f64(cuda):
    out = run([os.path.join(BIN, "anxrun"), "-np", "2", os.path.join(BIN, "anx_dgemm"), "1024", "--gpu"], 120)
    assert out.returncode == 0 and "Result verified" in out.stdout, out.stdout + out.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("algo", ["direct", "winograd"])
def test_convbench_all_layers(cuda, algo):
    out = run([os.path.join(BIN, "anx_convbench"), "--batch", "8", "--iters", "2", "--algo", algo], 300)
    assert out.returncode == 0, out.stderr
    lines = [l for l in out.stdout.splitlines() if "TFLOP/s" in l]
    assert len(lines) == 5 and all(l.endswith("OK") for l in lines), out.stdout


def test_lane_timeline_synthetic_trace(tmp_path):
    """tools/lane_timeline.py on a hand-made kernel trace: two queues whose kernels overlap, one 5 us idle
    gap; union, overlap, gaps and per-kernel medians come out as constructed."""
    import sys
    hdr = ('"Kind","Agent_Id","Queue_Id","Stream_Id","Thread_Id","Dispatch_Id","Kernel_Id","Kernel_Name",'
           '"Correlation_Id","Start_Timestamp","End_Timestamp"')
    rows = [  # (queue, name, start ns, end ns)
        (1, "conv1_fused_kernel<true>", 0, 100_000), (2, "gemm16_kernel<x>", 50_000, 150_000),
        (1, "pool_wino_in_kernel<4>", 155_000, 175_000), (2, "maxpool_lrn256_kernel<3>", 160_000, 170_000),
        (1, "__amd_rocclr_copyBuffer", 0, 500_000)]  # not a Blocks kernel: ignored
    p = tmp_path / "t.csv"
    p.write_text(hdr + "\n" + "\n".join(f'"KERNEL_DISPATCH","Agent 2",{q},0,1,{i},1,"{n}",{i},{s},{e}'
                                        for i, (q, n, s, e) in enumerate(rows)) + "\n")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "lane_timeline.py"), str(p)],
                         capture_output=True, text=True, check=True).stdout
    assert "window: 4 dispatches, 175.0 us wall" in out
    assert "any kernel running: 170.0 us" in out and "two or more: 60.0 us" in out
    assert "idle gaps: 1, total 5.0 us" in out
    assert "| `conv1_fused` | 1 | 100.0 | 100.0 |" in out
