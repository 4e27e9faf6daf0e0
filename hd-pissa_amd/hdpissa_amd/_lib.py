"""ctypes binding of libhdpissa.so (C-ABI declared in include/hdpissa.h).

The library is built in-tree (``make -C hd-pissa_amd``) into ``hdpissa_amd/_lib``.
``torch`` is imported first so that the library's DT_NEEDED ROCm runtimes
(libamdhip64.so.7, librccl.so.1, librocsolver.so.0, librocblas.so.5) bind to the copies
torch already loaded -- one HIP runtime per process.  There is no fallback: if the
library is missing every HIP op raises ``HdpLibraryError``.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must be loaded before the library, see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("HDPISSA_LIB", os.path.join(_HERE, "_lib", "libhdpissa.so"))

HDP_F32 = 0
HDP_BF16 = 1
HDP_DW_STORE = 0
HDP_DW_MERGE = 1
HDP_MATH_AUTO = 0
HDP_MATH_F32 = 1
HDP_MATH_X3 = 2
HDP_MATH_H2 = 3
HDP_X3_REGS, HDP_X3_GLDS, HDP_X3_WIDE = 0, 1, 2

_c_int, _c_i64, _c_f, _c_vp, _c_sz = ctypes.c_int, ctypes.c_int64, ctypes.c_float, ctypes.c_void_p, ctypes.c_size_t

class ProbeItem(ctypes.Structure):
    """hdp_probe_item (include/hdpissa.h)."""
    _fields_ = [("X", ctypes.c_void_p), ("G", ctypes.c_void_p), ("A", ctypes.c_void_p), ("B", ctypes.c_void_p),
                ("gA", ctypes.c_void_p), ("gB", ctypes.c_void_p), ("T", ctypes.c_int64), ("in_", ctypes.c_int64),
                ("out", ctypes.c_int64), ("r", ctypes.c_int), ("b_transposed", ctypes.c_int),
                ("accumulate", ctypes.c_int), ("scale", ctypes.c_float)]


class MergeItem(ctypes.Structure):
    """hdp_merge_item (include/hdpissa.h)."""
    _fields_ = [("W", ctypes.c_void_p), ("dW", ctypes.c_void_p), ("n", ctypes.c_int64)]


class SvdItem(ctypes.Structure):
    """hdp_svd_item (include/hdpissa.h)."""
    _fields_ = [("W", ctypes.c_void_p), ("out", ctypes.c_int64), ("in_", ctypes.c_int64), ("A_all", ctypes.c_void_p),
                ("B_all", ctypes.c_void_p), ("S", ctypes.c_void_p)]


class DeltaItem(ctypes.Structure):
    """hdp_delta_item (include/hdpissa.h)."""
    _fields_ = [("out", ctypes.c_int64), ("in_", ctypes.c_int64), ("r", ctypes.c_int), ("nseg", ctypes.c_int),
                ("dA", ctypes.c_void_p), ("dB", ctypes.c_void_p), ("delta_seg_stride", ctypes.c_int64),
                ("A", ctypes.c_void_p), ("B", ctypes.c_void_p), ("factor_seg_stride", ctypes.c_int64),
                ("dst", ctypes.c_void_p)]


# name -> (restype, argtypes); must match include/hdpissa.h exactly
SIGNATURES = {
    "hdp_abi_version": (_c_int, []),
    "hdp_last_error": (ctypes.c_char_p, []),
    "hdp_merge": (_c_int, [_c_vp, _c_int, _c_vp, _c_i64, _c_vp]),
    "hdp_merge_group": (_c_int, [_c_int, ctypes.POINTER(MergeItem), _c_int, _c_vp]),
    "hdp_merge_group_bf16dw": (_c_int, [_c_int, ctypes.POINTER(MergeItem), _c_vp]),
    "hdp_fold_bf16": (_c_int, [_c_vp, _c_int, _c_i64, _c_vp, _c_i64, _c_vp]),
    "hdp_adam_factors": (_c_int, [_c_vp, _c_vp, _c_vp, _c_vp, _c_i64, _c_f, _c_f, _c_f, _c_f, _c_f, _c_f,
                                  _c_f, _c_f, _c_f, _c_int, _c_vp]),
    "hdp_delta_gemm": (_c_int, [_c_i64, _c_i64, _c_int, _c_int, _c_vp, _c_vp, _c_i64, _c_vp, _c_vp, _c_i64,
                                _c_vp, _c_int, _c_int, _c_int, _c_vp]),
    "hdp_delta_set_math": (_c_int, [_c_int]),
    "hdp_delta_set_x3_stage": (_c_int, [_c_int]),
    "hdp_delta_plan_create": (_c_int, [ctypes.POINTER(DeltaItem), _c_int, _c_int, _c_int, _c_int,
                                       ctypes.POINTER(_c_vp)]),
    "hdp_delta_plan_run": (_c_int, [_c_vp, _c_vp]),
    "hdp_delta_plan_fused_adam": (_c_int, [_c_vp]),
    "hdp_delta_plan_run_adam": (_c_int, [_c_vp, _c_vp, _c_vp, _c_vp, _c_vp] + [ctypes.c_float] * 10 + [_c_int, _c_vp]),
    "hdp_delta_plan_fused_fallback": (_c_int, [_c_vp, ctypes.POINTER(_c_int)]),
    "hdp_delta_plan_invalidate": (_c_int, [_c_vp]),
    "hdp_delta_plan_tiles": (_c_int, [_c_vp, ctypes.POINTER(_c_i64), ctypes.POINTER(_c_int)]),
    "hdp_delta_plan_math": (_c_int, [_c_vp]),
    "hdp_delta_plan_destroy": (_c_int, [_c_vp]),
    "hdp_probe_workspace_bytes": (_c_sz, [_c_i64, _c_i64, _c_i64, _c_int]),
    "hdp_probe_grads": (_c_int, [_c_i64, _c_i64, _c_i64, _c_int, _c_vp, _c_vp, _c_int, _c_vp, _c_vp, _c_int,
                                 _c_vp, _c_vp, _c_f, _c_int, _c_vp, _c_sz, _c_vp]),
    "hdp_probe_group_max": (_c_int, []),
    "hdp_probe_errors": (_c_int, [_c_int]),
    "hdp_probe_host_wait_us": (_c_i64, [_c_int]),
    "hdp_probe_grads_group": (_c_int, [_c_int, ctypes.POINTER(ProbeItem), _c_int, _c_vp, _c_sz, _c_vp]),
    "hdp_probe_queue_create": (_c_int, [_c_int, _c_int, _c_i64, ctypes.POINTER(_c_vp)]),
    "hdp_probe_queue_add_module": (_c_int, [_c_vp, _c_vp, _c_vp, _c_int, _c_vp, _c_vp, _c_i64, _c_i64, _c_int, _c_f,
                                            ctypes.POINTER(_c_int)]),
    "hdp_probe_queue_push": (_c_int, [_c_vp, _c_int, _c_vp, _c_vp, _c_i64, _c_int, _c_vp, ctypes.POINTER(_c_int)]),
    "hdp_probe_queue_flush": (_c_int, [_c_vp]),
    "hdp_probe_queue_pending": (_c_int, [_c_vp]),
    "hdp_probe_queue_flushes": (_c_i64, [_c_vp]),
    "hdp_probe_queue_destroy": (_c_int, [_c_vp]),
    "hdp_svd_workspace_bytes": (_c_sz, [_c_i64, _c_i64, _c_int]),
    "hdp_svd_topk": (_c_int, [_c_vp, _c_int, _c_i64, _c_i64, _c_int, _c_int, _c_vp, _c_vp, _c_vp, _c_vp,
                              _c_sz, _c_vp]),
    "hdp_svd_batch_workspace_bytes": (_c_sz, [_c_int, ctypes.POINTER(SvdItem), _c_int]),
    "hdp_svd_topk_batched": (_c_int, [_c_int, ctypes.POINTER(SvdItem), _c_int, _c_int, _c_int, _c_vp, _c_sz, _c_vp]),
    "hdp_comm_unique_id": (_c_int, [_c_vp, _c_sz]),
    "hdp_comm_init": (_c_int, [ctypes.POINTER(_c_vp), _c_vp, _c_sz, _c_int, _c_int]),
    "hdp_comm_destroy": (_c_int, [_c_vp]),
    "hdp_allgather_f32": (_c_int, [_c_vp, _c_vp, _c_vp, _c_i64, _c_vp]),
    "hdp_allreduce_sum_f32": (_c_int, [_c_vp, _c_vp, _c_i64, _c_vp]),
    "hdp_broadcast_bytes": (_c_int, [_c_vp, _c_vp, _c_i64, _c_int, _c_vp]),
    "hdp_alltoall_f32": (_c_int, [_c_vp, _c_vp, _c_vp, _c_i64, _c_vp]),
    "hdp_allgather_bytes": (_c_int, [_c_vp, _c_vp, _c_vp, _c_i64, _c_vp]),
    "hdp_timing_enable": (_c_int, [_c_int]),
    "hdp_timing_reset": (_c_int, []),
    "hdp_timing_kernels": (_c_int, []),
    "hdp_timing_query": (_c_int, [_c_int, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(_c_i64),
                                  ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                  ctypes.POINTER(ctypes.c_double)]),
}


class HdpLibraryError(RuntimeError):
    pass


class HdpError(RuntimeError):
    pass


_lib = None


def lib() -> ctypes.CDLL:
    """Load (once) and return the library; raise ``HdpLibraryError`` if absent."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise HdpLibraryError(
                f"libhdpissa.so not found at {LIB_PATH}: build it with `make -C hd-pissa_amd` "
                "(or __graft_entry__.build()); there is no CPU fallback")
        L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if L.hdp_abi_version() != 1:
            raise HdpLibraryError("libhdpissa ABI version mismatch")
        _lib = L
    return _lib


def kernel_timing(enable=None, reset: bool = False) -> dict:
    """Live per-kernel HIP-event timing of this library's launches (hdp_timing_*).
    Returns {kernel: dict(launches, total_ms, avg_us, bytes_per_launch, flop_per_launch)}
    for the kernels launched since the last reset; ``enable`` switches recording on/off."""
    L = lib()
    out = {}
    for k in range(L.hdp_timing_kernels()):
        name, n = ctypes.c_char_p(), _c_i64()
        ms, by, fl = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        check(L.hdp_timing_query(k, ctypes.byref(name), ctypes.byref(n), ctypes.byref(ms), ctypes.byref(by),
                                 ctypes.byref(fl)), "hdp_timing_query")
        if n.value:
            out[name.value.decode()] = dict(launches=n.value, total_ms=ms.value, avg_us=1e3 * ms.value / n.value,
                                            bytes_per_launch=by.value / n.value, flop_per_launch=fl.value / n.value)
    if reset:
        check(L.hdp_timing_reset(), "hdp_timing_reset")
    if enable is not None:
        L.hdp_timing_enable(1 if enable else 0)
    return out


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = lib().hdp_last_error().decode(errors="replace")
        raise HdpError(f"{what} failed (status {rc}): {msg}")
