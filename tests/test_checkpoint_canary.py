"""Checkpoint round trips (safetensors + the raw format the native CLI reads) and the halo-canary
check of SURVEY §5.2: halo slots of every conv2 window are poisoned with NaN before the exchange; if
the planner missed a row that a tile needs, NaN reaches the output."""
import json
import os
import subprocess

import pytest
import torch

from anx.models.alexnet_blocks import AlexNetBlocks
from anx.parallel.plan import PER_LAYER, make_plan
from anx.utils.init import init_input, init_weights
from anx.utils.io import load_weights, load_weights_raw, save_weights, save_weights_raw

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ANX = os.path.join(ROOT, "cuda-mpi-gpu-cluster-programming_amd", "bin", "anx")


def test_safetensors_roundtrip(tmp_path):
    w = init_weights("rand", 9)
    save_weights(str(tmp_path / "w.safetensors"), w)
    r = load_weights(str(tmp_path / "w.safetensors"))
    assert all(torch.equal(w[k], r[k]) for k in w)


@pytest.mark.skipif(not os.path.exists(ANX), reason="native CLI not built")
def test_native_cli_reads_raw_checkpoint(tmp_path):
    w = init_weights("rand", 21)
    save_weights_raw(str(tmp_path), w)
    assert all(torch.equal(w[k], v) for k, v in load_weights_raw(str(tmp_path)).items())
    x = init_input(1, "const")
    ref = AlexNetBlocks(w, device="cpu")(x)
    out = subprocess.run([ANX, "--version", "v1", "--weights", str(tmp_path)], capture_output=True, text=True,
                         timeout=120)
    assert out.returncode == 0, out.stderr
    rec = json.loads(next(l for l in out.stdout.splitlines() if l.startswith("ANX_JSON"))[9:])
    import zlib
    assert rec["checksum"] == zlib.crc32(ref.numpy().tobytes()) & 0xFFFFFFFF


def _poisoned_per_layer(device, np_):
    m = AlexNetBlocks(device=device, init="rand", seed=13, max_batch=2)
    x = init_input(2, "rand", seed=13).to(device)
    full = m(x)
    p = make_plan(227, 227, np_, PER_LAYER)
    eng = [AlexNetBlocks(device=device, weights=m.weights, max_batch=2) for _ in range(np_)]
    for r, t in enumerate(p.tiles):
        if t.out.empty:
            continue
        eng[r].stage1(x[:, t.inp.lo:t.inp.hi].contiguous(), t)
        # poison every valid window row this tile did not compute itself (= must arrive as halo)
        for row in range(max(t.q.lo, 0), min(t.q.hi, 27)):
            if not (t.p1.lo <= row < t.p1.hi):
                eng[r].window_put(t, row, torch.full(eng[r].window_rows_shape(2, 1), float("nan"), device=device))
    for h in p.p1_halos:
        eng[h.dst].window_put(p.tiles[h.dst], h.rows.lo, eng[h.src].window_get(p.tiles[h.src], h.rows.lo, h.rows.hi, 2))
    out = torch.cat([eng[r].stage2(2, t) for r, t in enumerate(p.tiles) if not t.out.empty], dim=1)
    return out, full


@pytest.mark.parametrize("np_", [2, 3, 5, 8])
def test_halo_canary_cpu(np_):
    out, full = _poisoned_per_layer("cpu", np_)
    assert not torch.isnan(out).any()
    torch.testing.assert_close(out, full, rtol=0, atol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("np_", [2, 4, 8])
def test_halo_canary_gpu(cuda, np_):
    out, full = _poisoned_per_layer(cuda, np_)
    assert not torch.isnan(out).any()
    torch.testing.assert_close(out, full, rtol=1e-6, atol=1e-6)
