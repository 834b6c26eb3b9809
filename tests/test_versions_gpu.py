"""GPU staged versions on the MI355X: V3 golden values, V4 with 2 host-staged ranks sharing the
box's GPU (gloo comm, the reference's "all ranks on device 0" situation, D4), V5 single rank, and
--check against the fp64 oracle."""
import pytest

from test_versions_cpu import run_cli

pytestmark = pytest.mark.gpu


def test_v3_golden_raw(cuda):
    rec, out = run_cli(["--version", "v3", "--iters", "3"])
    assert "AlexNet HIP Forward Pass completed in" in out
    assert rec["first10"][:3] == pytest.approx([29.2932, 25.9153, 23.3255], abs=1e-3)
    assert rec["warm_ms"] is not None


def test_v3_batch_check(cuda):
    rec, _ = run_cli(["--version", "v3", "--batch", "16", "--init", "rand", "--check", "--iters", "2"])
    assert rec["max_abs_err"] < 1e-3


@pytest.mark.parametrize("extra", [[], ["--decomp", "per_layer"], ["--strategy", "batch"]])
def test_v4_two_ranks_one_gpu(cuda, extra):
    d = ["--conv2-algo", "direct", "--conv1-algo", "direct"]  # bit-identical across decompositions (Winograd: ~1e-7)
    ref, _ = run_cli(["--version", "v3", "--init", "rand", "--seed", "5", "--batch", "3", *d])
    rec, out = run_cli(["--version", "v4", "--init", "rand", "--seed", "5", "--batch", "3", *extra, *d], 2)
    assert "Final Output Shape: 13x13x256" in out
    assert rec["checksum"] == ref["checksum"]


def test_v5_single_rank(cuda):
    rec, _ = run_cli(["--version", "v5", "--init", "rand", "--check", "--batch", "4"])
    assert rec["max_abs_err"] < 1e-3


def test_v4_filter_parallel_two_ranks_one_gpu(cuda):
    """P7 filter split on GPU ranks (host-staged channel halo + gather) vs the fp64 oracle."""
    rec, out = run_cli(["--version", "v4", "--strategy", "filter", "--init", "rand", "--check", "--batch", "3"], 2)
    assert "Final Output Shape: 13x13x256" in out
    assert rec["max_abs_err"] < 1e-3
