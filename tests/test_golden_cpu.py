"""Golden-value tests on the C++ host engine, and host engine vs the PyTorch
fp64 oracle. The reference only ever eyeballed "first 5 values" (SURVEY §4); here they are
asserted, together with the full output tensor."""
import pytest
import torch

from anx.models.alexnet_blocks import AlexNetBlocks
from anx.models.reference import blocks_forward
from anx.utils.init import init_input

# final_project/logs/run_20250509_112555_DESKTOP-B5PMJB5/run_v2_2.1_broadcast_all_np1.log:2
GOLD_DIV_N = [44.4152, 42.4612, 40.6967, 40.6967, 40.6967]
# final_project/logs/run_20250509_112555_DESKTOP-B5PMJB5/run_v3_np1.log:2
GOLD_RAW = [29.2932, 25.9153, 23.3255, 23.3255, 23.3255]


@pytest.mark.parametrize("mode,gold", [("div_n", GOLD_DIV_N), ("raw", GOLD_RAW)])
def test_golden_first5(mode, gold):
    m = AlexNetBlocks(device="cpu", lrn_mode=mode)
    y = m(init_input(1, "const"))
    assert tuple(y.shape) == (1, 13, 13, 256)
    assert y.flatten()[:5].tolist() == pytest.approx(gold, abs=2e-4)


@pytest.mark.parametrize("mode", ["div_n", "raw"])
def test_host_engine_matches_torch_oracle(mode):
    m = AlexNetBlocks(device="cpu", init="rand", seed=3, lrn_mode=mode)
    x = init_input(2, "rand", seed=3)
    y = m(x)
    ref = blocks_forward(x, m.weights, m.b1, m.b2)
    torch.testing.assert_close(y.double(), ref, rtol=1e-5, atol=1e-6)


def test_grouped_conv2_matches_oracle():
    m = AlexNetBlocks(device="cpu", init="rand", seed=5, groups2=2)
    x = init_input(1, "rand", seed=5)
    torch.testing.assert_close(m(x).double(), blocks_forward(x, m.weights, m.b1, m.b2), rtol=1e-5, atol=1e-6)


def test_out_tensor_is_checked():
    """The engines write through the raw output pointer: a caller-supplied ``out`` of the wrong shape,
    dtype or layout is rejected before any native call (forward, forward_async, tile_forward, stage2)."""
    import pytest
    import torch

    from anx.models.alexnet_blocks import AlexNetBlocks, full_plan
    from anx.utils.init import init_input

    m = AlexNetBlocks(init="rand", seed=5, device="cpu")
    x = init_input(1, "rand", seed=5)
    good = m(x).clone()
    plan = full_plan(m.H, m.W, m.b1, m.b2)
    for bad in (torch.empty(1, 13, 13, 255), torch.empty(2, 13, 13, 256), torch.empty(1, 13, 13, 256, dtype=torch.float64),
                torch.empty(1, 13, 256, 13).transpose(2, 3)):
        with pytest.raises(ValueError):
            m(x, out=bad)
        with pytest.raises(ValueError):
            m.forward_async(x, bad)
        with pytest.raises(ValueError):
            m.tile_forward(x, plan, out=bad)
    y = torch.empty(1, 13, 13, 256)
    m.forward_async(x, y)
    m.join()
    assert torch.equal(y, good)


def test_oracle_all_images_chunked():
    """blocks_forward_all (the whole-batch fp64 oracle of the GPU tests and smoke) equals the one-call
    oracle image for image, across chunk boundaries (to fp64 rounding)."""
    from anx.models.reference import blocks_forward_all
    from anx.utils.init import init_weights
    w = init_weights("rand", 3)
    x = torch.rand(5, 67, 67, 3) * 0.1  # small images: conv1 15x15 -> pool 7 -> conv2 7 -> pool 3
    ref = blocks_forward(x, w)
    got = blocks_forward_all(x, w, chunk=2)
    assert got.dtype == torch.float64 and got.shape == ref.shape
    torch.testing.assert_close(got, ref, rtol=1e-12, atol=1e-14)  # fp64: the batch split may reorder sums
