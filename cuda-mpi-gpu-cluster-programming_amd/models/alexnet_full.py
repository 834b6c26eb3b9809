"""Full AlexNet (extension model family, BASELINE.json config "Full AlexNet Conv1-5 + FC6-8 bf16,
batch=2048"): the reference's Blocks 1-2 (Conv1-ReLU-Pool1-Conv2-ReLU-Pool2-LRN2) followed by the
AlexNet tail Conv3/4/5 (3x3, pad 1) + Pool5 + FC6/FC7/FC8, inference in bf16 with fp32 accumulation
on v_mfma_f32_32x32x16_bf16 (csrc/src/hip/conv_bf16.hip, csrc/src/full_engine.cpp).

The reference itself stops after Block 2; this family exists because the benchmark
configs name it. FC layers run on the same implicit-GEMM kernel as 1x1 convolutions.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch
import torch.nn.functional as F

from .. import _native as nat
from ..utils.init import STREAM_EXTRA, uniform
from ..utils.tuning import apply_knobs, knob_value

LAYERS = ("conv1", "conv2", "conv3", "conv4", "conv5", "fc6", "fc7", "fc8")
FLOPS_PER_IMAGE = 2.0 * (55 * 55 * 96 * 363 + 27 * 27 * 256 * 2400 + 13 * 13 * 384 * 2304 + 13 * 13 * 384 * 3456 +
                         13 * 13 * 256 * 3456 + 9216 * 4096 + 4096 * 4096 + 4096 * 1000)


def weight_shapes(classes: int = 1000, groups2: int = 1):
    wn, bn = (C.c_size_t * 8)(), (C.c_size_t * 8)()
    nat.call("anx_full_weight_sizes", classes, groups2, wn, bn)
    conv = [(96, 3, 11, 11), (256, 96 // groups2, 5, 5), (384, 256, 3, 3), (384, 384, 3, 3), (256, 384, 3, 3)]
    fc = [(4096, 9216), (4096, 4096), (classes, 4096)]
    shapes = conv + fc
    assert [int(np.prod(s)) for s in shapes] == list(wn)
    return shapes, [int(b) for b in bn]


def init_full_weights(seed: int = 0, classes: int = 1000, groups2: int = 1) -> dict:
    """He-uniform weights from the counter-based RNG (deterministic on every rank), zero biases."""
    shapes, bsz = weight_shapes(classes, groups2)
    out = {}
    for i, (name, s) in enumerate(zip(LAYERS, shapes)):
        fan_in = int(np.prod(s[1:]))
        bound = float(np.sqrt(6.0 / fan_in))
        u = uniform(seed, STREAM_EXTRA + i, int(np.prod(s)))
        out["w_" + name] = torch.from_numpy(((u * 2 - 1) * bound).astype(np.float32).reshape(s))
        out["b_" + name] = torch.zeros(bsz[i])
    return out


class AlexNetFull:
    def __init__(self, weights: dict | None = None, *, seed: int = 0, classes: int = 1000, device="cuda",
                 max_batch: int = 1, groups2: int = 1, lrn_mode: str = "div_n", knobs: dict | None = None,
                 lanes: int = 1):
        self.classes, self.groups2, self.lrn_mode = classes, groups2, lrn_mode
        self.knobs = {k: knob_value(k, v) for k, v in (knobs or {}).items()}  # e.g. {"bf16_glds": 3}
        self.weights = {k: v.detach().to("cpu", torch.float32).contiguous()
                        for k, v in (weights or init_full_weights(seed, classes, groups2)).items()}
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise ValueError("the bf16 full-AlexNet engine is GPU-only (use reference_forward on the CPU)")
        self._h = None
        self._cap = 0
        if lanes < 1:
            raise ValueError("lanes must be >= 1")
        per_lane = -(-max(1, max_batch) // lanes)
        self._ensure(per_lane)  # lane 0's share; a forward of more images on lane 0 alone grows it
        # lanes > 1: the batch is split over engines on concurrent HIP streams (forked from / joined to
        # the caller's stream, as AlexNetBlocks does), so one lane's partial last rounds overlap the
        # other's kernels. Measured slower at 256 images (281k vs 305k img/s: half-size launches of
        # the 1-workgroup-per-CU kernels quantize worse), 334k at 512 as 2 x 256
        # (profiles/r02_ab_full_lanes.txt)
        self._lanes: list[AlexNetFull] = []
        self._lane_streams: list[torch.cuda.Stream] = []
        for _ in range(lanes - 1):
            self._lanes.append(AlexNetFull(self.weights, classes=classes, device=self.device, max_batch=per_lane,
                                           groups2=groups2, lrn_mode=lrn_mode, knobs=self.knobs))
            self._lane_streams.append(torch.cuda.Stream(self.device))

    def _ensure(self, n):
        """Grow THIS engine to n images (the other lanes' engines are untouched)."""
        if self._h is not None and n <= self._cap:
            return
        if self._h is not None:
            torch.cuda.synchronize(self.device)
            nat.bf16().anx_full_destroy(self._h)
            self._h = None
        ws = (C.c_void_p * 8)(*[self.weights["w_" + k].data_ptr() for k in LAYERS])
        bs = (C.c_void_p * 8)(*[self.weights["b_" + k].data_ptr() for k in LAYERS])
        h = C.c_void_p()
        with torch.cuda.device(self.device):
            nat.call("anx_full_create", C.byref(h), ws, bs, self.classes, max(1, n), self.groups2,
                     0 if self.lrn_mode == "div_n" else 1)
        try:
            apply_knobs(h, self.knobs, full=True)
        except Exception:
            nat.bf16().anx_full_destroy(h)
            raise
        self._h, self._cap = h, max(1, n)

    def set_knob(self, name: str, value) -> None:
        v = knob_value(name, value)
        apply_knobs(self._h, {name: v}, full=True)
        self.knobs[name] = v
        for m in getattr(self, "_lanes", ()):
            m.set_knob(name, v)

    def close(self):
        for m in getattr(self, "_lanes", ()):
            m.close()
        if self._h is not None:
            torch.cuda.synchronize(self.device)
            nat.bf16().anx_full_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def _check(self, x: torch.Tensor, out: torch.Tensor | None) -> torch.Tensor:
        """The engine reads x and writes out through raw pointers: both must be exactly what the
        kernels assume (shape, dtype, contiguity, device)."""
        if (x.dim() != 4 or tuple(x.shape[1:]) != (227, 227, 3) or x.dtype != torch.float32 or not x.is_contiguous()
                or x.device != self.device):
            raise ValueError(f"expected contiguous fp32 NHWC [N,227,227,3] on {self.device}, got "
                             f"{tuple(x.shape)} {x.dtype} on {x.device}")
        shape = (x.shape[0], self.classes)
        if out is None:
            return torch.empty(shape, device=self.device)
        if (tuple(out.shape) != shape or out.dtype != torch.float32 or not out.is_contiguous()
                or out.device != self.device):
            raise ValueError(f"out must be a contiguous fp32 {shape} tensor on {self.device}, got "
                             f"{tuple(out.shape)} {out.dtype} on {out.device}")
        return out

    def forward(self, x: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        """x: [N,227,227,3] fp32 NHWC on the device -> logits [N, classes] fp32."""
        y = self._check(x, out)
        N = x.shape[0]
        L = 1 + len(self._lanes)
        if L == 1 or N < L:
            self._ensure(N)
            nat.call("anx_full_forward", self._h, x.data_ptr(), N, y.data_ptr(), nat.stream_ptr(self.device))
            return y
        bounds = [N * i // L for i in range(L + 1)]
        cur = torch.cuda.current_stream(self.device)
        for i, st in enumerate(self._lane_streams, start=1):
            st.wait_stream(cur)  # fork: inputs produced / outputs free on the current stream
            with torch.cuda.stream(st):
                self._lanes[i - 1].forward(x[bounds[i]:bounds[i + 1]], y[bounds[i]:bounds[i + 1]])
        self._ensure(bounds[1])
        nat.call("anx_full_forward", self._h, x.data_ptr(), bounds[1], y.data_ptr(), nat.stream_ptr(self.device))
        for st in self._lane_streams:
            cur.wait_stream(st)  # join
        return y

    __call__ = forward

    def forward_async(self, x: torch.Tensor, out: torch.Tensor, on_lane=None, pre_lane=None) -> torch.Tensor:
        """Throughput form for repeated forwards on the same buffers (contract of
        AlexNetBlocks.forward_async): lanes on their own streams, never joined per call; when all are
        idle they fork from the current stream and lane i starts at lane i-1's mid-forward mark
        (after Conv2 + Pool2/LRN), so they run half a forward apart. :meth:`join` before reading out."""
        out = self._check(x, out)
        N = x.shape[0]
        L = 1 + len(self._lanes)
        if L == 1 or N < L or self.device.type != "cuda":
            if pre_lane is not None:
                pre_lane(0, 0, N)
            self.forward(x, out)
            if on_lane is not None:
                on_lane(0, 0, N)
            return out
        if getattr(self, "_own_stream", None) is None:
            self._own_stream = torch.cuda.Stream(self.device)
        streams = [self._own_stream, *self._lane_streams]
        engines = [self, *self._lanes]
        bounds = self.lane_bounds(N)
        fresh = all(st.query() for st in streams)
        cur = torch.cuda.current_stream(self.device)
        for i, (eng, st) in enumerate(zip(engines, streams)):
            lo, hi = bounds[i], bounds[i + 1]
            eng._ensure(hi - lo)
            if fresh:
                st.wait_stream(cur)
                if i > 0:
                    nat.call("anx_full_wait_mark", engines[i - 1]._h, st.cuda_stream)
            fn = "anx_full_forward_mark" if fresh and i + 1 < L else "anx_full_forward"
            with torch.cuda.stream(st):
                if pre_lane is not None:
                    pre_lane(i, lo, hi)
                nat.call(fn, eng._h, x[lo:hi].data_ptr(), hi - lo, out[lo:hi].data_ptr(), st.cuda_stream)
                if on_lane is not None:
                    on_lane(i, lo, hi)
        return out

    def lane_bounds(self, n: int) -> list[int]:
        """Image boundaries [0, ..., n] of the lanes :meth:`forward_async` runs ``n`` images on (the
        pipeline's per-lane gather segments; ScatterComputeGather's root shedding needs them)."""
        L = 1 + len(self._lanes)
        if L == 1 or n < L or self.device.type != "cuda":
            return [0, n]
        return [n * i // L for i in range(L + 1)]

    def join(self) -> None:
        if self.device.type != "cuda":
            return
        cur = torch.cuda.current_stream(self.device)
        for st in [s for s in [getattr(self, "_own_stream", None)] if s is not None] + self._lane_streams:
            cur.wait_stream(st)

    TAPS = ((55, 55, 96), (31, 31, 96), (27, 27, 256), (15, 15, 256), (15, 15, 384), (15, 15, 384), (13, 13, 256),
            (9216,), (4096,), (4096,), (57, 57, 48))

    def tap(self, i: int, N: int) -> torch.Tensor:
        """bf16 activation ``i`` of the last forward (see FullEngine::tap): conv1, pool1 window,
        conv2, pool2+LRN window, conv3/conv4 windows, conv5, pool5, fc6, fc7; 10: the bf16
        polyphase (space-to-depth by 4) input of conv1. Tap 0 holds conv1 only when the forward
        wrote it: with pool1 fused into the Conv1 kernel (knob ``bf16_pool1``, one workgroup per
        image) the 55x55 map never leaves the kernel."""
        y = torch.empty((N, *self.TAPS[i]), device=self.device, dtype=torch.bfloat16)
        n = C.c_size_t()
        nat.call("anx_full_tap", self._h, i, N, y.data_ptr(), C.byref(n), nat.stream_ptr(self.device))
        return y


def reference_forward(x: torch.Tensor, w: dict, groups2: int = 1, lrn_mode: str = "div_n",
                      dtype=torch.float32) -> torch.Tensor:
    """Plain PyTorch oracle (NHWC in, logits out) of the same topology."""
    h = x.permute(0, 3, 1, 2).to(dtype)
    g = lambda k: w[k].to(h.device, dtype)  # noqa: E731
    h = F.max_pool2d(F.relu(F.conv2d(h, g("w_conv1"), g("b_conv1"), stride=4)), 3, 2)
    h = F.max_pool2d(F.relu(F.conv2d(h, g("w_conv2"), g("b_conv2"), padding=2, groups=groups2)), 3, 2)
    a = 1e-4 if lrn_mode == "div_n" else 1e-4 * 5
    h = F.local_response_norm(h, 5, alpha=a, beta=0.75, k=2.0)
    h = F.relu(F.conv2d(h, g("w_conv3"), g("b_conv3"), padding=1))
    h = F.relu(F.conv2d(h, g("w_conv4"), g("b_conv4"), padding=1))
    h = F.max_pool2d(F.relu(F.conv2d(h, g("w_conv5"), g("b_conv5"), padding=1)), 3, 2)
    h = h.permute(0, 2, 3, 1).reshape(h.shape[0], -1)  # NHWC flatten (the engine's FC6 input order)
    h = F.relu(F.linear(h, g("w_fc6"), g("b_fc6")))
    h = F.relu(F.linear(h, g("w_fc7"), g("b_fc7")))
    return F.linear(h, g("w_fc8"), g("b_fc8"))
