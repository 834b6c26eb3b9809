"""The cost model (anx/cost.hpp through anx.parallel.cost, no GPU): byte counts of every BASELINE
multi-GPU configuration pinned, the comm-aware row-split pick, and the modelled 1/2/4/8 curve's
contract (labelled as not measured; S and E as the reference's analytics define them,
/root/reference/log_analysis.py:212-222)."""
import os
import re
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from anx.parallel import cost  # noqa: E402

IN_IMG = 227 * 227 * 3 * 4      # 618,348 B
OUT_IMG = 13 * 13 * 256 * 4     # 173,056 B
IN_ROW = 227 * 3 * 4            # 2,724 B


def test_v5_root_egress_bytes():
    """The reference's V5 data flow (the root scatters 1024 images over 8 ranks every step): 554 MB of
    root egress for the batch split; a 2-way row split costs more: 673 MB with overlap tiles (147 / 131
    input rows) and 578 MB with per-layer tiles (123 / 115 rows)."""
    batch = cost.step("v5", 8, 1024, 1, input_source="root")["bytes"]
    assert batch["root_egress"] == 7 * 128 * IN_IMG  # 554.0 MB
    assert batch["max_peer_egress"] == 128 * IN_IMG
    assert batch["root_ingress"] == 7 * 128 * OUT_IMG  # 155.1 MB
    over = cost.step("v5", 8, 1024, 2, input_source="root", mode="overlap")["bytes"]
    assert over["root_egress"] == 256 * IN_ROW * (131 + 3 * (147 + 131))  # 672.9 MB
    per = cost.step("v5", 8, 1024, 2, input_source="root", mode="per_layer")["bytes"]
    assert per["root_egress"] == 256 * IN_ROW * (115 + 3 * (123 + 115))  # 578.1 MB
    assert per["max_rank_halo"] > 0 and batch["max_rank_halo"] == 0


def test_v5_local_input_moves_only_gather_and_halo():
    s = cost.step("v5", 8, 1024, 1, input_source="local")
    assert s["bytes"]["root_egress"] == 0 and s["egress_ms"] == 0
    assert s["bytes"]["root_ingress"] == 7 * 128 * OUT_IMG
    # round-6 kernels: 128 images per rank compute in about the time the root takes to receive the 7
    # peers' outputs, so the step sits at the compute / ingress balance point (never egress or halo)
    assert s["bound"] in ("compute", "ingress")
    assert s["ingress_ms"] <= 1.05 * s["compute_ms"] and s["halo_ms"] == 0
    # the root-scatter data flow is egress-bound at 8 ranks whatever the kernels do
    r = cost.step("v5", 8, 1024, -1, input_source="root")
    assert r["bound"] == "egress" and r["step_ms"] > 3 * s["step_ms"]


def test_v4_h2d_bytes_and_pick():
    """V4 at 4 ranks x 256 images is H2D-bound: the 2-way row split DMAs 51.3 MB on the busiest rank,
    the batch split 39.6 MB, so the model picks the batch split (V4 never needs rows here)."""
    rows = cost.step("v4", 4, 256, 2)
    batch = cost.step("v4", 4, 256, 1)
    assert rows["bytes"]["max_rank_h2d"] == 128 * 147 * IN_ROW  # 51.25 MB
    assert batch["bytes"]["max_rank_h2d"] == 64 * 227 * IN_ROW  # 39.57 MB
    assert batch["bound"] == "h2d" and batch["step_ms"] < rows["step_ms"]
    assert cost.pick_row_ways("v4", 4, 256) == 1


def test_pick_row_ways_v5():
    assert cost.pick_row_ways("v5", 8, 1024) == 1
    assert cost.pick_row_ways("v5", 1, 5) == 1
    # 2 images over 8 GPUs: every candidate is latency-bound (a forward never takes less than its
    # kernel chain), so the pick is the one with the least communication
    tiny = cost.step("v5", 8, 2)
    assert tiny["bound"] in ("compute", "halo") and tiny["compute_ms"] >= 0.08
    # the pick minimises the modelled step over the divisors of np
    for np_, batch in ((2, 64), (4, 8), (8, 1024), (8, 12)):
        best = min((cost.step("v5", np_, batch, r)["step_ms"], r) for r in range(1, np_ + 1) if np_ % r == 0)
        assert cost.step("v5", np_, batch, cost.pick_row_ways("v5", np_, batch))["step_ms"] == pytest.approx(best[0])


@pytest.mark.parametrize("wl,batch", [("dp", 128), ("v4", 256), ("v5", 1024)])
def test_curve_contract(wl, batch):
    c = cost.curve(wl, batch, input_source="root" if wl == "v4" else "local")
    assert c["measured"] is False and c["N"] == [1, 2, 4, 8]
    assert c["scaling"] == ("weak" if wl == "dp" else "strong")
    for i, n in enumerate(c["N"]):
        assert c["efficiency"][i] == pytest.approx(c["speedup"][i] / n, abs=2e-3)
        assert c["bound"][i] in ("compute", "egress", "ingress", "halo", "h2d", "d2h", "host")
    assert c["speedup"][0] == pytest.approx(1.0)
    step0 = c["steps"][0]
    imgs = batch if wl != "dp" else batch
    assert c["images_per_s"][0] == pytest.approx(imgs / step0["step_ms"] * 1e3, rel=1e-3)


def test_dp_ingest_and_overrides():
    """dp at 8 GPUs: rank 0 ingests 7 x 128 images of output per step (155 MB); with slower links the
    step turns ingress-bound, with a measured ingest slowdown the root's compute grows."""
    flat = {"ingest_slowdown": 0, "dp_root_shed": 0}
    s = cost.step("dp", 8, 128, overrides=flat)
    assert s["bytes"]["root_ingress"] == 7 * 128 * OUT_IMG
    slow = cost.step("dp", 8, 128, overrides=dict(flat, xgmi_gbps=20))
    assert slow["bound"] == "ingress" and slow["step_ms"] > s["step_ms"]
    probe = cost.step("dp", 8, 128, overrides={"ingest_slowdown": 0.1, "dp_root_shed": 0})
    # the slowdown is per 155.06 MB received per step: 7 x 128 images of output is that volume
    assert probe["compute_ms"] == pytest.approx(s["compute_ms"] * (1 + 0.1 * 7 * 128 * OUT_IMG / 155.06e6), rel=1e-3)
    two = cost.step("dp", 2, 128, overrides={"ingest_slowdown": 0.1, "dp_root_shed": 0})
    base2 = cost.step("dp", 2, 128, overrides=flat)
    assert two["compute_ms"] == pytest.approx(base2["compute_ms"] * (1 + 0.1 * 128 * OUT_IMG / 155.06e6), rel=1e-3)
    r = cost.curve("dp", 128, overrides="rate=64:100000,128:200000")
    assert r["images_per_s"][0] == pytest.approx(200000, rel=1e-6)
    with pytest.raises(Exception, match="unknown parameter"):
        cost.step("dp", 2, 128, overrides="nope=1")


def test_dp_root_shed():
    """dp: rank 0 computes B / (1 + its ingest slowdown) images (even), the peers B; the job's images
    per step and the modelled rate count the shed share."""
    assert cost.dp_root_batch(1, 128) == 128
    assert cost.dp_root_batch(8, 128) == 2 * round(128 / (1 + 0.15 * 7 * 128 * OUT_IMG / 155.06e6) / 2) == 112
    assert cost.dp_root_batch(8, 128, overrides="dp_root_shed=0") == 128
    assert cost.dp_root_batch(2, 128) == 126 and cost.dp_root_batch(8, 2) == 2
    s = cost.step("dp", 8, 128)
    assert s["root_batch"] == 112 and s["images"] == 7 * 128 + 112
    assert s["bytes"]["root_ingress"] == 7 * 128 * OUT_IMG  # peers still send full batches
    assert s["images_per_s"] == pytest.approx(s["images"] / s["step_ms"] * 1e3, rel=1e-3)
    noshed = cost.step("dp", 8, 128, overrides="dp_root_shed=0")
    assert noshed["root_batch"] == 128
    # at the ASSUMED 50 GB/s per xGMI link the round-6 kernels make the N=8 step ingress-bound (0.46 ms
    # gather vs 0.39 ms compute), where the shed costs 16 of 1024 images (1.6 %); when the link is faster
    # the step is compute-bound and the shed is what keeps rank 0 off the critical path (13 % of a step).
    # The bench keeps the shed: the cheap side of an unmeasurable link rate.
    assert s["bound"] == "ingress" and noshed["images_per_s"] < 1.02 * s["images_per_s"]
    fast = "xgmi_gbps=150"
    s, noshed = cost.step("dp", 8, 128, overrides=fast), cost.step("dp", 8, 128, overrides=fast + ";dp_root_shed=0")
    assert s["bound"] == "compute" and s["step_ms"] < noshed["step_ms"]
    assert s["images_per_s"] > noshed["images_per_s"]


def test_readme_scaling_section_is_the_model():
    """The README's modelled scaling tables are generated by tools/scaling_readme.py from this model."""
    from tools.scaling_readme import render
    with open(os.path.join(ROOT, "README.md")) as f:
        text = f.read()
    m = re.search(r"<!-- scaling-model:begin -->\n(.*?)<!-- scaling-model:end -->", text, re.S)
    assert m, "README lacks the generated scaling section"
    assert m.group(1) == render()


@pytest.mark.parametrize("np_,batch,rw", [(8, 1024, 1), (8, 1024, 2), (4, 256, 2), (2, 64, 2), (4, 6, 4)])
@pytest.mark.parametrize("src", ["root", "local"])
def test_model_bytes_are_the_runtime_schedule(np_, batch, rw, src):
    """The model's root egress / ingress and busiest-rank halo bytes equal the sums over the native V5
    runtime's own transfer schedule (libanx_dist record-only schedule; no GPU)."""
    from anx.parallel.workloads import native_schedule
    sched = native_schedule(np_, batch, rw, input_source=src)
    sent, recv = {}, {}
    egress = ingress = 0
    for l in sched:
        ph, edge, w, h = l.split(" ")[:4]
        s, d = (int(v) for v in edge.split("->"))
        if s == d:
            continue
        b = int(w[2:]) * int(h[2:])
        if ph.startswith("scatter"):
            egress += b
        elif ph.startswith("gather"):
            ingress += b
        else:
            sent[s] = sent.get(s, 0) + b
            recv[d] = recv.get(d, 0) + b
    m = cost.step("v5", np_, batch, rw, input_source=src)["bytes"]
    assert m["root_egress"] == egress and m["root_ingress"] == ingress
    assert m["max_rank_halo"] == max([0, *sent.values(), *recv.values()])
