"""bench.py's driver contract on one MI355X: one JSON line with the BASELINE metric and config, for
the headline Blocks 1-2 fp32 step (2 stream lanes) and the full-AlexNet bf16 extension."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config")


def bench(args):
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup", "1", *args],
                         capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert all(k in rec for k in KEYS) and rec["n_gpus"] == 1 and rec["steps"] == 3 and rec["value"] > 0
    return rec


@pytest.mark.gpu
def test_bench_blocks_contract():
    with open(os.path.join(ROOT, "BASELINE.json")) as f:
        metric = json.load(f)["metric"]
    rec = bench(["--batch-per-gpu", "64"])
    c = rec["config"]
    assert rec["metric"] == metric and rec["dtype"] == "fp32" and c["global_batch"] == 64
    assert c["lanes"] == 2 and rec["vs_baseline"] > 1 and c["b1_warm_ms"] > 0
    # vs_baseline is the like-for-like cold ratio (fresh process, one image), the warm one has its own key
    assert rec["vs_baseline"] == c["b1_process_cold_vs_reference"] and "cold" in rec["vs_baseline_kind"]
    assert c["b1_vs_reference_warm"] > rec["vs_baseline"]
    # unambiguous semantics: distinct input batches beyond the Infinity Cache, an engine-cold and a
    # process-cold (fresh `anx --version v3` process) batch-1 latency next to the reference's 610.661 ms
    assert c["input_batches_rotated"] >= 4 and c["input_bytes_rotated"] > (256 << 20)
    assert c["b1_engine_cold_ms"] > c["b1_warm_ms"] and "b1_cold_ms" not in c
    assert c["b1_process_cold_ms"] > c["b1_engine_cold_ms"] * 0.5 and c["b1_process_cold_vs_reference"] > 0
    trials = sorted(c["b1_process_cold_trials_ms"])  # the record is the median fresh process
    assert len(trials) == 3 and c["b1_process_cold_ms"] == trials[1] and c["b1_process_gap_s"] == 2.0
    assert c["gpu_max_hw_queues"] == "8"
    # the matrix-core work actually executed stays below the fp32 MFMA peak; the direct-convolution
    # equivalent may not (Winograd does 4x fewer multiplies)
    assert 0 < c["mfma_tflops"] < 160
    assert abs(c["direct_equiv_tflops"] / c["mfma_tflops"] - c["gflop_per_image_direct"] / c["gflop_per_image_mfma"]) < 0.05
    # BASELINE configs 3 / 4 beside the headline (native runtimes), the halo-on V5 arms on the shared GPU,
    # and the modelled curve outside config
    assert c["model"].startswith("AlexNet Blocks1-2") and rec["model_curve"]["measured"] is False
    v4, v5 = rec["v4"], rec["v5"]
    assert v4["auto"]["global_batch"] == 256 and v4["auto"]["images_per_s"] > 0 and "halo_exchange" in v4["auto"]
    assert v5["auto"]["global_batch"] == 1024 and v5["auto"]["images_per_s"] > 0 and v5["auto"]["output_crc"] != 0
    assert v5["rows2_peer"]["halo_bytes_per_step"] > 0 and v5["rows2_peer"]["outputs_match_loopback"] is True


@pytest.mark.gpu
@pytest.mark.parametrize("workload", ["v4", "v5"])
def test_bench_workloads_one_gpu(workload):
    rec = bench(["--workload", workload, "--batch", "16", "--no-b1"])
    c = rec["config"]
    assert rec["scaling"] == "strong" and c["global_batch"] == 16 and c["workload"] == workload
    if workload == "v4":  # the native host-staged runtime: chunked per-rank DMA, link rate reported
        assert c["phases_ms"]["compute"] > 0 and c["h2d_gbps_link"] > 1 and 0 < c["h2d_bound_fraction"] < 1.5
        assert c["chunks"] >= 1 and c["runtime"].startswith("native")
        assert "RCCL" not in c["pipeline"] and "per-rank chunked H2D" in c["pipeline"]
    else:  # the native runtime: critical-path phases, balanced layout, transport
        assert c["phases_ms"]["stage2"] > 0 and c["transport"] == "rccl" and c["imbalance"] == 1.0
        # the halo-on sub-records: both device transports, the same output bit for bit
        peer, loop = rec["v5_rows2_peer"], rec["v5_rows2_loopback"]
        assert peer["halo_bytes_per_step"] > 0 and loop["checksum"] is not None
        assert peer["outputs_match_loopback"] is True


@pytest.mark.gpu
def test_bench_v5_peer_transport_one_gpu():
    """bench.py --workload v5 --transport peer (the IPC transport with device-side flags) at N=1."""
    rec = bench(["--workload", "v5", "--transport", "peer", "--batch", "32", "--no-b1"])
    c = rec["config"]
    assert c["transport"] == "peer" and c["ordering"] == "flags" and c["phases_ms"]["stage2"] > 0


@pytest.mark.gpu
def test_bench_full_contract():
    rec = bench(["--model", "full", "--batch-per-gpu", "32"])
    assert rec["dtype"] == "bf16" and rec["config"]["global_batch"] == 32
