"""Per-layer operators on torch tensors (NHWC fp32), each one native kernel.

GPU tensors run the libanx HIP kernels on torch's current stream; CPU tensors run libanx's C++ host
reference kernels. There is no eager-PyTorch path (the torch oracle is anx.models.reference).
These are the standalone, testable layer ops of SURVEY §7.1 item 3. They match the reference's
per-layer kernels:

* convKernel / serialConvLayer  (v3_cuda_only/src/layers_cuda.cu:20-46, v1_serial/src/layers_serial.cpp:37-81)
* reluKernel                    (layers_cuda.cu:56-62)
* poolKernel                    (layers_cuda.cu:78-104)
* lrnKernel                     (layers_cuda.cu:118-152; alpha mode: ``div_n`` V1/V2, ``raw`` V3/V4)

How the GPU versions differ:

* ``conv2d`` is the MFMA implicit GEMM: packed weights are cached per (weight tensor, version, plan).
  The cache entry holds a reference to the weight tensor, so its storage (and address) cannot be
  reused by another tensor while the entry exists; in-place edits through ``w.data`` do not bump
  ``w._version`` — call :func:`clear_cache` after them. ``impl="direct"`` selects the
  one-thread-per-output oracle kernel.
* ``maxpool`` uses float4 channels.
* ``maxpool_lrn`` is the fused pool+LRN kernel.
* ``conv2d`` can write into a channel slice of a preallocated output (``out`` / ``c_off``), which
  is how the filter-parallel strategy assembles its shards.
"""
from __future__ import annotations

import ctypes as C

import torch
import torch.nn.functional as F

from .. import _native as nat
from ..config import conv_out_dim, pool_out_dim

__all__ = ["conv2d", "relu", "maxpool", "lrn", "maxpool_lrn", "clear_cache"]

_LRN_MODES = {"div_n": 0, "raw": 1}
_pack_cache: dict = {}


def clear_cache() -> None:
    _pack_cache.clear()


def _check(x: torch.Tensor, name: str) -> None:
    if x.dtype != torch.float32 or not x.is_contiguous():
        raise ValueError(f"{name}: expected a contiguous float32 tensor")


def _packed(w: torch.Tensor, plan, sizes: tuple[int, int], dev: torch.device):
    key = (w.data_ptr(), w._version, tuple(w.shape), w.stride(), str(w.device), tuple(plan), str(dev))
    hit = _pack_cache.get(key)
    if hit is not None and hit[0] is w:
        return hit[1], hit[2]
    wc = w.detach().to("cpu", torch.float32).contiguous()
    packed = torch.empty(sizes[0], dtype=torch.float32)
    koff = torch.empty(sizes[1], dtype=torch.int32)
    nat.call("anx_conv_pack", plan, C.c_void_p(wc.data_ptr()), C.c_void_p(packed.data_ptr()),
             C.c_void_p(koff.data_ptr()))
    if len(_pack_cache) > 64:
        _pack_cache.clear()
    # keep `w` alive with the entry: a freed temporary's address could otherwise be handed to the
    # next temporary of the same shape (e.g. equal-size filter shards) and hit this entry
    hit = (w, packed.to(dev), koff.to(dev))
    _pack_cache[key] = hit
    return hit[1], hit[2]


def conv2d(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None = None, stride: int = 1, pad: int = 0,
           groups: int = 1, relu: bool = False, impl: str = "mfma", out: torch.Tensor | None = None,
           c_off: int = 0) -> torch.Tensor:
    """x [N,H,W,C], w [K,C/groups,F,F] (KCFF), b [K] -> [N,Ho,Wo,K] (or into out[..., c_off:c_off+K])."""
    _check(x, "conv2d")
    N, H, W, Cin = x.shape
    K, Cg, Fh, Fw = w.shape
    if Fh != Fw or Cg * groups != Cin or K % groups:
        raise ValueError("conv2d: bad weight shape")
    Ho, Wo = conv_out_dim(H, Fh, stride, pad), conv_out_dim(W, Fw, stride, pad)
    if out is None:
        out = torch.empty((N, Ho, Wo, K), device=x.device, dtype=torch.float32)
        c_off = 0
    if out.shape[:3] != (N, Ho, Wo) or c_off + K > out.shape[3]:
        raise ValueError("conv2d: out has the wrong shape")
    _check(out, "conv2d out")
    bias = (b if b is not None else torch.zeros(K, device=x.device)).to(x.device, torch.float32).contiguous()
    if not x.is_cuda:
        if c_off or out.shape[3] != K:
            tmp = torch.empty((N, Ho, Wo, K), dtype=torch.float32)
            conv2d(x, w, bias, stride, pad, groups, relu, impl, tmp)
            out[..., c_off:c_off + K] = tmp
            return out
        wc = w.detach().float().contiguous()
        nat.call("anx_cpu_conv2d", nat.ptr(x), nat.ptr(wc), nat.ptr(bias), nat.ptr(out), N, H, W, Cin, K, Fh,
                 stride, pad, groups, int(relu))
        return out
    s = nat.stream_ptr(x.device)
    if impl == "direct":
        if c_off or out.shape[3] != K:
            raise ValueError("conv2d: impl='direct' writes whole outputs only")
        wd = w.detach().to(x.device, torch.float32).contiguous()
        nat.call("anx_conv2d_direct", nat.ptr(x), nat.ptr(wd), nat.ptr(bias), nat.ptr(out), N, H, W, Cin, K, Fh,
                 stride, pad, groups, int(relu), s)
        return out
    xp = F.pad(x, (0, 0, pad, pad, pad, pad)).contiguous() if pad else x
    plan = (C.c_int * 16)()
    sz, kz = C.c_size_t(), C.c_size_t()
    nat.call("anx_conv_plan", N, H + 2 * pad, W + 2 * pad, Cin, K, Fh, stride, groups, plan, C.byref(sz), C.byref(kz))
    packed, koff = _packed(w, plan, (sz.value, kz.value), x.device)
    nat.call("anx_conv2d_mfma", plan, nat.ptr(xp), nat.ptr(packed), nat.ptr(koff), nat.ptr(bias), nat.ptr(out),
             Ho, Wo, out.shape[3], 0, 0, c_off, int(relu), s)
    return out


def relu(x: torch.Tensor, inplace: bool = False) -> torch.Tensor:
    _check(x, "relu")
    y = x if inplace else x.clone()
    if y.is_cuda:
        nat.call("anx_relu", nat.ptr(y), y.numel(), nat.stream_ptr(y.device))
    else:
        y.clamp_(min=0.0)  # host ReLU is part of anx_cpu_conv2d (relu=True); standalone it is one clamp
    return y


def maxpool(x: torch.Tensor, size: int = 3, stride: int = 2, impl: str = "vec4") -> torch.Tensor:
    _check(x, "maxpool")
    N, H, W, Cn = x.shape
    Ho, Wo = pool_out_dim(H, size, stride), pool_out_dim(W, size, stride)
    y = torch.empty((N, Ho, Wo, Cn), device=x.device, dtype=torch.float32)
    if not x.is_cuda:
        nat.call("anx_cpu_maxpool", nat.ptr(x), nat.ptr(y), N, H, W, Cn, size, stride)
    elif impl == "direct" or Cn % 4:
        nat.call("anx_maxpool_direct", nat.ptr(x), nat.ptr(y), N, H, W, Cn, size, stride, nat.stream_ptr(x.device))
    else:
        nat.call("anx_maxpool", nat.ptr(x), N, H, W, Cn, size, stride, nat.ptr(y), Ho, Wo, Cn, 0, 0, 0,
                 nat.stream_ptr(x.device))
    return y


def lrn(x: torch.Tensor, size: int = 5, alpha: float = 1e-4, beta: float = 0.75, k: float = 2.0,
        mode: str = "div_n") -> torch.Tensor:
    _check(x, "lrn")
    N, H, W, Cn = x.shape
    y = torch.empty_like(x)
    m = _LRN_MODES[mode]
    if x.is_cuda:
        nat.call("anx_lrn_direct", nat.ptr(x), nat.ptr(y), N, H, W, Cn, size, alpha, beta, k, m,
                 nat.stream_ptr(x.device))
    else:
        nat.call("anx_cpu_lrn", nat.ptr(x), nat.ptr(y), N, H, W, Cn, size, alpha, beta, k, m)
    return y


def maxpool_lrn(x: torch.Tensor, pool: int = 3, stride: int = 2, size: int = 5, alpha: float = 1e-4,
                beta: float = 0.75, k: float = 2.0, mode: str = "div_n") -> torch.Tensor:
    """Fused max-pool + LRN (one kernel on the GPU; pool then LRN on the host)."""
    _check(x, "maxpool_lrn")
    if not x.is_cuda or x.shape[3] % 4:
        return lrn(maxpool(x, pool, stride), size, alpha, beta, k, mode)
    N, H, W, Cn = x.shape
    y = torch.empty((N, pool_out_dim(H, pool, stride), pool_out_dim(W, pool, stride), Cn), device=x.device)
    nat.call("anx_maxpool_lrn", nat.ptr(x), nat.ptr(y), N, H, W, Cn, pool, stride, size, alpha, beta, k,
             _LRN_MODES[mode], nat.stream_ptr(x.device))
    return y
