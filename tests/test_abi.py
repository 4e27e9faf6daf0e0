"""The C-ABI library loads on a CPU-only host and exports every symbol include/hdpissa.h
declares; the ctypes table covers exactly that set.  No compute calls (no GPU here)."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "hdpissa.h")


def declared_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(hdp_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_the_api():
    syms = declared_symbols()
    for s in ("hdp_merge", "hdp_adam_factors", "hdp_delta_gemm", "hdp_probe_grads", "hdp_svd_topk",
              "hdp_comm_init", "hdp_allgather_f32", "hdp_allreduce_sum_f32", "hdp_last_error"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    from hdpissa_amd._lib import LIB_PATH, SIGNATURES, lib
    if not os.path.exists(LIB_PATH):
        pytest.skip("libhdpissa.so not built (run __graft_entry__.build())")
    L = lib()
    for s in declared_symbols():
        assert hasattr(L, s), s
    assert sorted(SIGNATURES) == declared_symbols()
    assert L.hdp_abi_version() == 1


def test_argument_validation_without_gpu():
    """Host-side validation runs before any HIP call, so it is testable on CPU."""
    from hdpissa_amd._lib import LIB_PATH, lib
    if not os.path.exists(LIB_PATH):
        pytest.skip("libhdpissa.so not built")
    L = lib()
    assert L.hdp_delta_gemm(0, 4, 4, 1, None, None, 0, None, None, 0, None, 0, 1, 0, None) == 1
    assert b"bad shape" in L.hdp_last_error()
    assert L.hdp_merge(None, 7, None, 4, None) == 1
    assert L.hdp_probe_grads(4, 4, 4, 200, None, None, 0, None, None, 0, None, None, 1.0, 0, None, 0, None) == 1
    assert b"r = 200" in L.hdp_last_error()
    assert L.hdp_svd_topk(None, 0, 8, 8, 4, 4, None, None, None, None, 0, None) == 1
    assert b"exceeds" in L.hdp_last_error()
    import ctypes
    from hdpissa_amd._lib import DeltaItem
    items = (DeltaItem * 1)()
    items[0].out, items[0].in_, items[0].r, items[0].nseg = 8, 8, 0, 1
    h = ctypes.c_void_p()
    assert L.hdp_delta_plan_create(items, 1, 0, 1, 0, ctypes.byref(h)) == 1 and not h.value
    assert b"bad shape" in L.hdp_last_error()
    assert L.hdp_delta_plan_run(None, None) == 1
    assert L.hdp_delta_plan_destroy(None) == 0
    assert L.hdp_probe_workspace_bytes(1024, 4096, 4096, 16) > 0
    assert L.hdp_svd_workspace_bytes(4096, 4096, 16) >= 2 * 8 * 4096 * 4096


def test_torch_binding_loads_without_gpu():
    """hdpissa_amd._C (the torch binding of the native probe queue) loads against the in-tree
    libhdpissa.so and creates / destroys a queue without touching a GPU."""
    import torch  # noqa: F401
    from hdpissa_amd import _C
    q = _C.ProbeQueue(False, 8, 1 << 20)
    assert q.pending() == 0 and q.flushes() == 0 and q.handle() != 0
    q.close()
    with pytest.raises(RuntimeError):
        _C.ProbeQueue(False, 100000, 1 << 20)  # max_items beyond hdp_probe_group_max()
