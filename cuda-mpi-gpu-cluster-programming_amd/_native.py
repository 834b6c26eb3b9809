"""ctypes binding of libanx (the native C++/HIP core, csrc/).

libanx.so is built in-tree (``python __graft_entry__.py`` or ``cmake -B build && ninja -C build``)
into ``lib/`` next to this file. It NEEDs ``libamdhip64.so.7``; when torch is imported first the
loader resolves that soname to torch's own HIP runtime, so the kernels run on torch's device
context and streams.

On a machine with a GPU the native library is mandatory: ``lib()`` raises if it is missing or
fails to load, so nothing silently falls back to eager PyTorch. On a CPU-only machine the CPU
reference paths still need it (they are C++ too); pure-Python oracles live in
``anx.models.reference``.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import torch  # noqa: F401  (load torch's HIP runtime before libanx)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ANX_LIB", os.path.join(_HERE, "lib", "libanx.so"))
DIST_PATH = os.path.join(os.path.dirname(LIB_PATH), "libanx_dist.so")
BF16_PATH = os.path.join(os.path.dirname(LIB_PATH), "libanx_bf16.so")

_lock = threading.Lock()
_lib = None
_dist = None


class BlockC(C.Structure):
    _fields_ = [
        ("C", C.c_int), ("K", C.c_int), ("F", C.c_int), ("S", C.c_int), ("P", C.c_int), ("groups", C.c_int),
        ("pool_F", C.c_int), ("pool_S", C.c_int),
        ("has_lrn", C.c_int), ("lrn_N", C.c_int),
        ("lrn_alpha", C.c_float), ("lrn_beta", C.c_float), ("lrn_k", C.c_float),
        ("lrn_mode", C.c_int),
    ]


class TileC(C.Structure):
    _fields_ = [(n, C.c_int) for n in (
        "in_lo", "in_hi", "c1_lo", "c1_hi", "p1_lo", "p1_hi", "q_lo", "q_hi", "c2_lo", "c2_hi", "out_lo", "out_hi")]


class XferC(C.Structure):
    _fields_ = [("src", C.c_int), ("dst", C.c_int), ("lo", C.c_int), ("hi", C.c_int)]


_P = C.c_void_p
_I = C.c_int
_F = C.c_float
_SZ = C.c_size_t

_SIGS = {
    "anx_last_error": (C.c_char_p, []),
    "anx_abi_version": (_I, []),
    "anx_device_count": (_I, []),
    "anx_default_blocks": (None, [C.POINTER(BlockC), C.POINTER(BlockC)]),
    "anx_make_plan": (_I, [_I, _I, _I, _I, C.POINTER(BlockC), C.POINTER(BlockC), C.POINTER(TileC), C.POINTER(_I),
                           C.POINTER(_I), C.POINTER(XferC), C.POINTER(_I), C.POINTER(XferC), C.POINTER(_I), _I]),
    "anx_make_hybrid_plan": (_I, [_I, _I, _I, _I, _I, _I, C.POINTER(BlockC), C.POINTER(BlockC), C.POINTER(_I),
                                  C.POINTER(_I), C.POINTER(_I), C.POINTER(_I), C.POINTER(_I), C.POINTER(TileC),
                                  C.POINTER(C.c_double)]),
    "anx_channel_copy": (_I, [_P, _P, _SZ, _I, _P]),
    "anx_cost_curve": (_I, [_I, C.POINTER(_I), _I, _I, _I, _I, _I, C.c_char_p, C.c_char_p, _SZ]),
    "anx_cost_step": (_I, [_I, _I, _I, _I, _I, _I, C.c_char_p, C.c_char_p, _SZ]),
    "anx_cost_pick_row_ways": (_I, [_I, _I, _I, _I, _I, C.c_char_p, C.POINTER(_I)]),
    "anx_cost_dp_root_batch": (_I, [_I, _I, C.c_char_p, C.POINTER(_I)]),
    "anx_engine_create": (_I, [C.POINTER(_P), C.POINTER(BlockC), C.POINTER(BlockC), _I, _I, _P, _P, _P, _P, _I, _I]),
    "anx_engine_destroy": (_I, [_P]),
    "anx_engine_forward": (_I, [_P, _P, _I, _P, _P]),
    "anx_engine_tile_forward": (_I, [_P, _P, _I, C.POINTER(TileC), _P, _P]),
    "anx_engine_stage1": (_I, [_P, _P, _I, C.POINTER(TileC), _P]),
    "anx_engine_stage2": (_I, [_P, _I, C.POINTER(TileC), _P, _P]),
    "anx_engine_window": (_I, [_P, C.POINTER(TileC), _I, _I, C.POINTER(_P), C.POINTER(_SZ), C.POINTER(_SZ)]),
    "anx_cpu_engine_create": (_I, [C.POINTER(_P), C.POINTER(BlockC), C.POINTER(BlockC), _I, _I, _P, _P, _P, _P]),
    "anx_cpu_engine_destroy": (_I, [_P]),
    "anx_cpu_engine_tile_forward": (_I, [_P, _P, _I, C.POINTER(TileC), _P]),
    "anx_cpu_engine_stage1": (_I, [_P, _P, _I, C.POINTER(TileC)]),
    "anx_cpu_engine_stage2": (_I, [_P, _I, C.POINTER(TileC), _P]),
    "anx_cpu_engine_window": (_I, [_P, C.POINTER(TileC), _I, _I, C.POINTER(_P), C.POINTER(_SZ), C.POINTER(_SZ)]),
    "anx_memcpy2d_host": (_I, [_P, _SZ, _P, _SZ, _SZ, _SZ]),
    "anx_memcpy2d_async": (_I, [_P, _SZ, _P, _SZ, _SZ, _SZ, _P]),
    "anx_conv2d_direct": (_I, [_P, _P, _P, _P] + [_I] * 10 + [_P]),
    "anx_relu": (_I, [_P, _SZ, _P]),
    "anx_maxpool_direct": (_I, [_P, _P] + [_I] * 6 + [_P]),
    "anx_lrn_direct": (_I, [_P, _P, _I, _I, _I, _I, _I, _F, _F, _F, _I, _P]),
    "anx_maxpool": (_I, [_P] + [_I] * 6 + [_P] + [_I] * 6 + [_P]),
    "anx_maxpool_lrn": (_I, [_P, _P] + [_I] * 6 + [_I, _F, _F, _F, _I, _P]),
    "anx_conv_plan": (_I, [_I] * 8 + [C.POINTER(_I), C.POINTER(_SZ), C.POINTER(_SZ)]),
    "anx_conv_pack": (_I, [C.POINTER(_I), _P, _P, _P]),
    "anx_conv1_wino": (_I, [_P, _I, _I, _I, _P, _I, _I, _P, _P, _I, _P]),
    "anx_conv2_wino": (_I, [_P, _I, _I, _I, _I, _P, _I, _I, _P, _P, _I, _P]),
    "anx_conv2_wino_tile": (_I, [_P, _I, _I, _I, _I, _P, _I, _I, _P, _P, _I, _P, _I]),
    "anx_engine_set_knob": (_I, [_P, C.c_char_p, _I]),
    "anx_engine_get_knob": (_I, [_P, C.c_char_p, C.POINTER(_I)]),
    "anx_default_knob": (_I, [C.c_char_p, C.POINTER(_I)]),
    "anx_conv2d_mfma": (_I, [C.POINTER(_I), _P, _P, _P, _P, _P] + [_I] * 6 + [_I, _P]),
    "anx_cpu_conv2d": (_I, [_P, _P, _P, _P] + [_I] * 10),
    "anx_cpu_maxpool": (_I, [_P, _P] + [_I] * 6),
    "anx_cpu_lrn": (_I, [_P, _P, _I, _I, _I, _I, _I, _F, _F, _F, _I]),
    "anx_cpu_blocks_forward": (_I, [C.POINTER(BlockC), C.POINTER(BlockC), _I, _I, _P, _P, _P, _P, _P, _I, _P]),
    "anx_rng_uniform": (_I, [C.c_uint64, C.c_uint64, _P, _SZ]),
}


_DIST_SIGS = {
    "anx_v5_create": (_I, [C.POINTER(_P), _I, _I, _I, _I, _I, C.c_char_p, _I, C.c_double, C.POINTER(BlockC),
                           C.POINTER(BlockC), _I, _I, _P, _P, _P, _P, _I, _I, _I, C.c_char_p, _I, _I, _I, _I,
                           C.c_char_p, _I, _I, _I, _I]),
    "anx_v5_log": (_I, [_P, C.c_char_p, _SZ]),
    "anx_v5_destroy": (_I, [_P]),
    "anx_v5_set_input": (_I, [_P, _P]),
    "anx_v5_step": (_I, [_P, _I]),
    "anx_v5_sync": (_I, [_P]),
    "anx_v5_output": (_I, [_P, _P]),
    "anx_v5_phases": (_I, [_P, C.c_char_p, _SZ, _I]),
    "anx_v5_describe": (_I, [_P, C.c_char_p, _SZ]),
    "anx_v4_create": (_I, [C.POINTER(_P), _I, _I, _I, _I, _I, C.c_char_p, _I, C.c_double, C.POINTER(BlockC),
                           C.POINTER(BlockC), _I, _I, _P, _P, _P, _P, _I, _I, _I, _I]),
    "anx_v4_destroy": (_I, [_P]),
    "anx_v4_segment": (_I, [_P, _P, _P]),
    "anx_v4_input_ready": (_I, [_P]),
    "anx_v4_step": (_I, [_P, _I]),
    "anx_v4_sync_all": (_I, [_P]),
    "anx_v4_phases": (_I, [_P, C.c_char_p, _SZ, _I]),
    "anx_v4_describe": (_I, [_P, C.c_char_p, _SZ]),
    "anx_v4_probe_h2d": (_I, [_P, _I, C.POINTER(C.c_double)]),
    "anx_v5_schedule": (_I, [_I, C.POINTER(BlockC), C.POINTER(BlockC), _I, _I, _I, _I, _I, _I, _I, C.c_char_p,
                             _I, C.c_char_p, _SZ]),
}


class NativeError(RuntimeError):
    pass


def available() -> bool:
    try:
        lib()
        return True
    except NativeError:
        return False


# libanx_bf16: the full-AlexNet bf16 engine (its own library, loaded on first use)
_BF16_SIGS = {
    "anx_full_weight_sizes": (_I, [_I, _I, C.POINTER(_SZ), C.POINTER(_SZ)]),
    "anx_full_create": (_I, [C.POINTER(_P), C.POINTER(_P), C.POINTER(_P), _I, _I, _I, _I]),
    "anx_full_destroy": (_I, [_P]),
    "anx_full_forward": (_I, [_P, _P, _I, _P, _P]),
    "anx_full_forward_mark": (_I, [_P, _P, _I, _P, _P]),
    "anx_full_wait_mark": (_I, [_P, _P]),
    "anx_full_set_knob": (_I, [_P, C.c_char_p, _I]),
    "anx_full_tap": (_I, [_P, _I, _I, _P, C.POINTER(_SZ), _P]),
    "anx_full_get_knob": (_I, [_P, C.c_char_p, C.POINTER(_I)]),
}
_bf16 = None


def lib():
    """The loaded libanx (raises NativeError if it cannot be loaded)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise NativeError(f"libanx not built: {LIB_PATH} missing (run `python __graft_entry__.py build`)")
        try:
            h = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
        except OSError as e:  # pragma: no cover - depends on the machine
            raise NativeError(f"cannot load {LIB_PATH}: {e}") from e
        for name, (res, args) in _SIGS.items():
            fn = getattr(h, name)
            fn.restype = res
            fn.argtypes = args
        _lib = h
        return _lib


def dist():
    """libanx_dist (the V5 multi-GPU runtime's C ABI; needs RCCL, so loaded only when used)."""
    global _dist
    if _dist is not None:
        return _dist
    lib()  # libanx first: libanx_dist links against it and reports errors through anx_last_error
    with _lock:
        if _dist is not None:
            return _dist
        if not os.path.exists(DIST_PATH):
            raise NativeError(f"libanx_dist not built: {DIST_PATH} missing (run `python __graft_entry__.py build`)")
        try:
            h = C.CDLL(DIST_PATH, mode=C.RTLD_GLOBAL)
        except OSError as e:  # pragma: no cover - depends on the machine
            raise NativeError(f"cannot load {DIST_PATH}: {e}") from e
        for name, (res, args) in _DIST_SIGS.items():
            fn = getattr(h, name)
            fn.restype = res
            fn.argtypes = args
        _dist = h
        return _dist


def dist_call(name: str, *args) -> None:
    check(getattr(dist(), name)(*args), name)


def bf16():
    """libanx_bf16 (the bf16 full-AlexNet engine; loaded only when a full model is built)."""
    global _bf16
    if _bf16 is not None:
        return _bf16
    lib()  # libanx first: libanx_bf16 links against it and reports errors through anx_last_error
    with _lock:
        if _bf16 is not None:
            return _bf16
        if not os.path.exists(BF16_PATH):
            raise NativeError(f"libanx_bf16 not built: {BF16_PATH} missing (run `python __graft_entry__.py build`)")
        try:
            h = C.CDLL(BF16_PATH, mode=C.RTLD_GLOBAL)
        except OSError as e:  # pragma: no cover - depends on the machine
            raise NativeError(f"cannot load {BF16_PATH}: {e}") from e
        for name, (res, args) in _BF16_SIGS.items():
            fn = getattr(h, name)
            fn.restype = res
            fn.argtypes = args
        _bf16 = h
        return _bf16


def check(status: int, what: str = "") -> None:
    if status != 0:
        msg = lib().anx_last_error().decode(errors="replace")
        raise NativeError(f"{what}: {msg}" if what else msg)


def call(name: str, *args) -> None:
    check(getattr(bf16() if name in _BF16_SIGS else lib(), name)(*args), name)


def ptr(t) -> int:
    """Raw data pointer of a torch tensor (must be contiguous)."""
    if not t.is_contiguous():
        raise ValueError("native ops need contiguous tensors")
    return t.data_ptr()


def stream_ptr(device=None) -> int:
    """hipStream_t of torch's current stream on `device`."""
    return torch.cuda.current_stream(device).cuda_stream


def block_c(spec) -> BlockC:
    """anx.config.BlockSpec -> BlockC."""
    c, p, l = spec.conv, spec.pool, spec.lrn
    return BlockC(c.C, c.K, c.F, c.S, c.P, c.groups, p.F, p.S, int(spec.has_lrn), l.N, l.alpha, l.beta, l.k,
                  0 if l.mode == "div_n" else 1)
