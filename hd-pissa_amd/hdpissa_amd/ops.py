"""Tensor-level wrappers of the HIP kernels (the default, and only shipped, op set).

Every method validates devices/dtypes/shapes on the host, then calls the C-ABI on torch's
*current* HIP stream.  Tensors are passed as raw device pointers; views into arenas are
allowed (their ``data_ptr`` is the segment-0 start).  There is no CPU path: a tensor that
is not on a HIP device raises.
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch

from . import _lib
from ._lib import HDP_BF16, HDP_F32, check, lib


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _dt(t: torch.Tensor) -> int:
    if t.dtype == torch.float32:
        return HDP_F32
    if t.dtype == torch.bfloat16:
        return HDP_BF16
    raise TypeError(f"unsupported dtype {t.dtype} (float32 / bfloat16 only)")


def _need_gpu(*ts):
    for t in ts:
        if not t.is_cuda:
            raise RuntimeError("hdpissa_amd HIP ops need tensors on a HIP device (no CPU fallback)")


def _f32(*ts):
    for t in ts:
        if t.dtype != torch.float32:
            raise TypeError(f"expected float32, got {t.dtype}")


class HipOps:
    """The MI355X kernel set (libhdpissa.so)."""

    name = "hip"

    def __init__(self):
        lib()  # fail loudly now if the library is missing
        self._ws = {}

    # -- scratch (stream-ordered reuse on the current stream) -----------------------------
    def _workspace(self, key: str, nbytes: int, device) -> torch.Tensor:
        buf = self._ws.get((key, device))
        if buf is None or buf.numel() < nbytes:
            buf = torch.empty(max(nbytes, 256), dtype=torch.uint8, device=device)
            self._ws[(key, device)] = buf
        return buf

    def release_workspace(self, key: str) -> None:
        """Drop a cached scratch buffer (e.g. the batched SVD's, ~4 GB, once the init is done)."""
        for k in [k for k in self._ws if k[0] == key]:
            del self._ws[k]

    # -- K1 --------------------------------------------------------------------------------
    def svd_topk(self, W: torch.Tensor, r: int, nranks: int) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        """Top r*nranks singular triplets of W -> (A_all [k, in], B_all [nranks, out, r], S [k])."""
        _need_gpu(W)
        W = W.contiguous()
        out, inn = W.shape
        k = r * nranks
        if k > min(out, inn):
            raise ValueError(f"ranks_per_gpu * world_size = {k} exceeds min(out, in) = {min(out, inn)}")
        A_all = torch.empty(k, inn, dtype=torch.float32, device=W.device)
        B_all = torch.empty(nranks, out, r, dtype=torch.float32, device=W.device)
        S = torch.empty(k, dtype=torch.float64, device=W.device)
        nb = lib().hdp_svd_workspace_bytes(out, inn, k)
        ws = self._workspace("svd", nb, W.device)
        check(lib().hdp_svd_topk(W.data_ptr(), _dt(W), out, inn, r, nranks, A_all.data_ptr(), B_all.data_ptr(),
                                 S.data_ptr(), ws.data_ptr(), ws.numel(), _stream()), "hdp_svd_topk")
        return A_all, B_all, S

    @staticmethod
    def _svd_chunk(Ws, idx, k: int, budget_bytes: int) -> int:
        """Items per hdp_svd_topk_batched call so that the library's workspace stays within
        ``budget_bytes``: the per-item cost is the library's own count (Gram, eigen-solver arrays, the
        block-Krylov basis / products / projection when that path runs, the projection buffer), taken
        as the workspace of three items minus two at the group's largest shape (a single item also
        holds the dsyevdx buffer).  rocSOLVER's internal dsyevd workspace (owned by its handle) is on
        top of it."""
        from ._lib import SvdItem
        big = max(idx, key=lambda i: max(Ws[i].shape))
        out, inn = Ws[big].shape

        def ws(count):
            arr = (SvdItem * count)()
            for j in range(count):
                arr[j].out, arr[j].in_ = out, inn
            return int(lib().hdp_svd_batch_workspace_bytes(count, arr, k))
        two = ws(2)
        per = max(ws(3) - two, 1)
        if budget_bytes < two:
            return 1
        return 2 + int((budget_bytes - two) // per)

    def svd_topk_batch(self, Ws, r: int, nranks: int, budget_bytes: Optional[int] = None):
        """svd_topk over many matrices: those sharing (dtype, min(out, in)) are batched through one
        strided-batched eigensolve per workspace-sized chunk (hdp_svd_topk_batched).  Returns the
        per-matrix (A_all, B_all, S) in input order."""
        import ctypes
        import os
        from ._lib import SvdItem
        if budget_bytes is None:
            budget_bytes = int(float(os.environ.get("HDP_SVD_BATCH_MB", "4096")) * (1 << 20))
        k = r * nranks
        res = [None] * len(Ws)
        groups = {}
        for i, W in enumerate(Ws):
            _need_gpu(W)
            if k > min(W.shape):
                raise ValueError(f"ranks_per_gpu * world_size = {k} exceeds min(out, in) = {min(W.shape)}")
            groups.setdefault((W.dtype, min(W.shape), W.device), []).append(i)
        for (dtype, n, dev), idx in groups.items():
            chunk = self._svd_chunk(Ws, idx, k, budget_bytes)
            for c0 in range(0, len(idx), chunk):
                part = idx[c0:c0 + chunk]
                arr = (SvdItem * len(part))()
                keep = []
                for j, i in enumerate(part):
                    W = Ws[i].contiguous()
                    out, inn = W.shape
                    A_all = torch.empty(k, inn, dtype=torch.float32, device=dev)
                    B_all = torch.empty(nranks, out, r, dtype=torch.float32, device=dev)
                    S = torch.empty(k, dtype=torch.float64, device=dev)
                    it = arr[j]
                    it.W, it.out, it.in_ = W.data_ptr(), out, inn
                    it.A_all, it.B_all, it.S = A_all.data_ptr(), B_all.data_ptr(), S.data_ptr()
                    keep.append(W)
                    res[i] = (A_all, B_all, S)
                nb = lib().hdp_svd_batch_workspace_bytes(len(part), arr, k)
                ws = self._workspace("svd", nb, dev)
                check(lib().hdp_svd_topk_batched(len(part), arr, _dt(keep[0]), r, nranks, ws.data_ptr(), ws.numel(),
                                                 _stream()), "hdp_svd_topk_batched")
        return res

    # -- K2 --------------------------------------------------------------------------------
    def probe_grads(self, X: torch.Tensor, G: torch.Tensor, A: torch.Tensor, B: torch.Tensor,
                    gA: torch.Tensor, gB: torch.Tensor, scale: float, accumulate: bool,
                    Bt: Optional[torch.Tensor] = None) -> None:
        """gA (+)= scale (G B)^T X; gB (+)= scale G^T (X A^T).  ``Bt`` (r x out, = B^T) lets the
        kernel read B with 16-byte row loads; B itself is then only used for shape checks."""
        _need_gpu(X, G, A, B, gA, gB)
        _f32(A, B, gA, gB)
        if X.dtype != G.dtype:
            raise TypeError("X and G must share the model dtype")
        T, inn = X.shape
        out = G.shape[1]
        r = A.shape[0]
        if G.shape[0] != T or A.shape[1] != inn or B.shape != (out, r) or gA.shape != A.shape or gB.shape != B.shape:
            raise ValueError("probe_grads: shape mismatch")
        for t in (X, G, A, B, gA, gB):
            if not t.is_contiguous():
                raise ValueError("probe_grads: tensors must be contiguous")
        if Bt is not None:
            _need_gpu(Bt)
            _f32(Bt)
            if Bt.shape != (r, out) or not Bt.is_contiguous():
                raise ValueError("probe_grads: Bt must be a contiguous r x out tensor")
        nb = lib().hdp_probe_workspace_bytes(T, inn, out, r) if T > 0 else 0
        ws = self._workspace("probe", nb, X.device)
        Bp, btr = (Bt, 1) if Bt is not None else (B, 0)
        check(lib().hdp_probe_grads(T, inn, out, r, X.data_ptr(), G.data_ptr(), _dt(X), A.data_ptr(), Bp.data_ptr(),
                                    btr, gA.data_ptr(), gB.data_ptr(), float(scale), int(bool(accumulate)),
                                    ws.data_ptr(), ws.numel(), _stream()), "hdp_probe_grads")

    def probe_errors(self, clear: bool = False) -> int:
        """The probe's device error word (a sweep hand-off wait gave up in a completed launch):
        host-mapped, read without synchronising (hdp_probe_errors)."""
        return int(lib().hdp_probe_errors(int(bool(clear))))

    def probe_group_max(self) -> int:
        return int(lib().hdp_probe_group_max())

    def probe_grads_group(self, items) -> None:
        """items: list of (X, G, A, Bt, gA, gB, scale, accumulate) -- one grouped launch per
        pass (same r-block and dtype; distinct gradients).  Bt is B^T (r x out)."""
        if not items:
            return
        from ._lib import ProbeItem
        n = len(items)
        arr = (ProbeItem * n)()
        dt = _dt(items[0][0])
        total = 0
        for i, (X, G, A, Bt, gA, gB, scale, acc) in enumerate(items):
            T, inn = X.shape
            out = G.shape[1]
            r = A.shape[0]
            if not (X.is_cuda and G.is_cuda and gA.is_cuda and gB.is_cuda):
                raise RuntimeError("hdpissa_amd HIP ops need tensors on a HIP device (no CPU fallback)")
            if X.dtype != G.dtype or _dt(X) != dt:
                raise TypeError("probe group: X and G must share one model dtype")
            if G.shape[0] != T or A.shape[1] != inn or Bt.shape != (r, out) or gA.shape != (r, inn) \
                    or gB.shape != (out, r):
                raise ValueError("probe group: shape mismatch")
            it = arr[i]
            it.X, it.G, it.A, it.B = X.data_ptr(), G.data_ptr(), A.data_ptr(), Bt.data_ptr()
            it.gA, it.gB = gA.data_ptr(), gB.data_ptr()
            it.T, it.in_, it.out, it.r = T, inn, out, r
            it.b_transposed, it.accumulate, it.scale = 1, int(bool(acc)), float(scale)
            total += lib().hdp_probe_workspace_bytes(T, inn, out, r) if T > 0 else 0
        ws = self._workspace("probe", total, items[0][0].device)
        check(lib().hdp_probe_grads_group(n, arr, dt, ws.data_ptr(), ws.numel(), _stream()),
              "hdp_probe_grads_group")

    def probe_group_raw(self, carr, n: int, X0: torch.Tensor, ws_bytes: int, stream: int) -> None:
        """Launch a prefilled ctypes ProbeItem array (the ProbeQueue fast path)."""
        ws = self._workspace("probe", ws_bytes, X0.device)
        check(lib().hdp_probe_grads_group(n, carr, _dt(X0), ws.data_ptr(), ws.numel(), stream),
              "hdp_probe_grads_group")

    # -- K3 --------------------------------------------------------------------------------
    def adam(self, grad: torch.Tensor, m: torch.Tensor, v: torch.Tensor, delta: torch.Tensor, t: int, lr: float,
             beta1: float, beta2: float, eps: float, zero_grad: bool, grad_scale: float = 1e16) -> None:
        _need_gpu(grad, m, v, delta)
        _f32(grad, m, v, delta)
        n = grad.numel()
        if not (m.numel() == v.numel() == delta.numel() == n):
            raise ValueError("adam: size mismatch")
        s = adam_scalars(t, lr, beta1, beta2, eps, grad_scale)
        check(lib().hdp_adam_factors(grad.data_ptr(), m.data_ptr(), v.data_ptr(), delta.data_ptr(), n, *s,
                                     int(bool(zero_grad)), _stream()), "hdp_adam_factors")

    # -- K4 --------------------------------------------------------------------------------
    def delta_gemm(self, out: int, inn: int, r: int, nseg: int, dA: torch.Tensor, dB: torch.Tensor,
                   delta_stride: int, A: torch.Tensor, B: torch.Tensor, factor_stride: int, dst: torch.Tensor,
                   mode: int, round_bf16: bool) -> None:
        _need_gpu(dA, dB, A, B, dst)
        _f32(dA, dB, A, B)
        if dst.numel() < out * inn or not dst.is_contiguous():
            raise ValueError("delta_gemm: dst must be a contiguous out x in tensor")
        for t, stride in ((dA, delta_stride), (dB, delta_stride), (A, factor_stride), (B, factor_stride)):
            need = (nseg - 1) * stride + r * (inn if t is dA or t is A else out)
            if t.storage_offset() + need > t.untyped_storage().nbytes() // 4:
                raise ValueError("delta_gemm: segment range exceeds the operand storage")
        check(lib().hdp_delta_gemm(out, inn, r, nseg, dA.data_ptr(), dB.data_ptr(), delta_stride, A.data_ptr(),
                                   B.data_ptr(), factor_stride, dst.data_ptr(), _dt(dst), mode, int(bool(round_bf16)),
                                   _stream()), "hdp_delta_gemm")

    def delta_plan(self, items, mode: int, round_bf16: bool) -> "DeltaPlan":
        """Grouped persistent K4 over many modules (one launch per run()).  items: list of
        (out, inn, r, nseg, dA, dB, delta_stride, A, B, factor_stride, dst) exactly as
        delta_gemm takes them; the plan keeps the tensors alive and captures their pointers."""
        return DeltaPlan(items, mode, round_bf16)

    # -- K5 --------------------------------------------------------------------------------
    def merge(self, W: torch.Tensor, dW: torch.Tensor) -> None:
        _need_gpu(W, dW)
        _f32(dW)
        if W.numel() != dW.numel() or not W.is_contiguous() or not dW.is_contiguous():
            raise ValueError("merge: W and dW must be contiguous with equal sizes")
        check(lib().hdp_merge(W.data_ptr(), _dt(W), dW.data_ptr(), W.numel(), _stream()), "hdp_merge")


    def merge_group(self, pairs) -> None:
        """K5 over many (W, dW) pairs (one exchange bucket) in one launch per dtype run.  dW is
        float32, or bfloat16 for bf16 W (the rank-ordered bf16 exchange: W = bf16(W + dW))."""
        from ._lib import MergeItem
        runs = []
        for W, dW in pairs:
            _need_gpu(W, dW)
            if dW.dtype == torch.bfloat16 and W.dtype != torch.bfloat16:
                raise TypeError("merge_group: a bfloat16 dW needs a bfloat16 W")
            if dW.dtype != torch.bfloat16:
                _f32(dW)
            if W.numel() != dW.numel() or not W.is_contiguous() or not dW.is_contiguous():
                raise ValueError("merge_group: W and dW must be contiguous with equal sizes")
            key = (W.dtype, dW.dtype)
            if not runs or runs[-1][0] != key:
                runs.append((key, []))
            runs[-1][1].append((W, dW))
        for (wdt, ddt), run in runs:
            arr = (MergeItem * len(run))()
            for i, (W, dW) in enumerate(run):
                arr[i].W, arr[i].dW, arr[i].n = W.data_ptr(), dW.data_ptr(), W.numel()
            if ddt == torch.bfloat16:
                check(lib().hdp_merge_group_bf16dw(len(run), arr, _stream()), "hdp_merge_group_bf16dw")
            else:
                check(lib().hdp_merge_group(len(run), arr, _dt(run[0][0]), _stream()), "hdp_merge_group")

    def fold_bf16(self, parts: torch.Tensor, out: torch.Tensor) -> None:
        """Rank-ordered bf16 fold (hp:389-392 rounding order): parts [nparts, n] float32 (rank i's
        term -bracket_i in row i), out [n] bfloat16 = bf16(...bf16(bf16(0 + p0) + p1)... + p_last)."""
        _need_gpu(parts, out)
        _f32(parts)
        if out.dtype != torch.bfloat16 or parts.dim() != 2 or out.numel() != parts.shape[1]:
            raise ValueError("fold_bf16: parts [nparts, n] float32 and out [n] bfloat16")
        if parts.stride(1) != 1 or not out.is_contiguous():
            raise ValueError("fold_bf16: rows of parts and out must be contiguous")
        check(lib().hdp_fold_bf16(parts.data_ptr(), parts.shape[0], parts.stride(0), out.data_ptr(), out.numel(),
                                  _stream()), "hdp_fold_bf16")


class DeltaPlan:
    """Owner of an hdp_delta_plan (C-ABI): descriptors of every item uploaded once; run()
    launches the grouped kernel on the current stream.  The captured tensors are held, and
    run() refuses to launch if any of them was re-allocated (e.g. a replaced W_res)."""

    def __init__(self, items, mode: int, round_bf16: bool):
        import ctypes
        from ._lib import DeltaItem
        if not items:
            raise ValueError("delta_plan: no items")
        n = len(items)
        arr = (DeltaItem * n)()
        dt = None
        self._tensors = []
        for i, (out, inn, r, nseg, dA, dB, dstr, A, B, fstr, dst) in enumerate(items):
            _need_gpu(dA, dB, A, B, dst)
            _f32(dA, dB, A, B)
            d = _dt(dst)
            if dt is None:
                dt = d
            elif d != dt:
                raise TypeError("delta_plan: all destinations must share one dtype")
            if dst.numel() < out * inn or not dst.is_contiguous():
                raise ValueError("delta_plan: dst must be a contiguous out x in tensor")
            for t, stride in ((dA, dstr), (dB, dstr), (A, fstr), (B, fstr)):
                need = (nseg - 1) * stride + r * (inn if t is dA or t is A else out)
                if t.storage_offset() + need > t.untyped_storage().nbytes() // 4:
                    raise ValueError("delta_plan: segment range exceeds the operand storage")
            it = arr[i]
            it.out, it.in_, it.r, it.nseg = out, inn, r, nseg
            it.dA, it.dB, it.delta_seg_stride = dA.data_ptr(), dB.data_ptr(), dstr
            it.A, it.B, it.factor_seg_stride = A.data_ptr(), B.data_ptr(), fstr
            it.dst = dst.data_ptr()
            self._tensors.append((dst, dst.data_ptr(), dA, dB, A, B))
        h = ctypes.c_void_p()
        check(lib().hdp_delta_plan_create(arr, n, dt, int(mode), int(bool(round_bf16)), ctypes.byref(h)),
              "hdp_delta_plan_create")
        self._h = h
        self._lib = lib()
        self.n = n
        # one tensor per distinct factor storage (A / B are views of an arena: views share their base's
        # version counter, so an in-place write to any factor -- load_state_dict, a re-init -- bumps it)
        reps = {}
        for _, _, _, _, A, B in self._tensors:
            for t in (A, B):
                reps.setdefault(t.untyped_storage().data_ptr(), t)
        self._factor_reps = list(reps.values())
        self._factor_versions = None

    def valid(self, dsts=None) -> bool:
        """True while every captured destination still has its captured storage."""
        if dsts is None:
            return all(t.data_ptr() == p for t, p, *_ in self._tensors)
        return all(d.data_ptr() == p for d, (_, p, *_r) in zip(dsts, self._tensors))

    def tiles(self):
        import ctypes
        t, g = ctypes.c_int64(), ctypes.c_int()
        check(self._lib.hdp_delta_plan_tiles(self._h, ctypes.byref(t), ctypes.byref(g)), "hdp_delta_plan_tiles")
        return t.value, g.value

    def math(self) -> str:
        """The MFMA math of the plan: 'f32', 'x3' or 'h2' (its roofline basis)."""
        return {1: "f32", 2: "x3", 3: "h2"}.get(int(self._lib.hdp_delta_plan_math(self._h)), "?")

    def run(self) -> None:
        check(self._lib.hdp_delta_plan_run(self._h, _stream()), "hdp_delta_plan_run")
        self._factor_versions = None  # (run re-packs every panel; the next run_adam re-packs the constants)

    def invalidate(self) -> None:
        """Re-pack the constant operand halves on the next run_adam (factors rewritten in place)."""
        check(self._lib.hdp_delta_plan_invalidate(self._h), "hdp_delta_plan_invalidate")

    def fused_adam(self) -> bool:
        """Adam folds into this plan's operand preparation (single-segment H2 merge plans)."""
        return bool(self._lib.hdp_delta_plan_fused_adam(self._h))

    def run_adam(self, grad: torch.Tensor, m: torch.Tensor, v: torch.Tensor, delta: torch.Tensor, t: int, lr: float,
                 beta1: float, beta2: float, eps: float, zero_grad: bool, grad_scale: float = 1e16) -> None:
        """K3 over the plan's factor entries folded into its K4 run (hp:356-373 + hp:389-394): the
        arenas' bases (the items' dA / dB point into ``delta``); m, v, delta as ``adam`` computes them."""
        _need_gpu(grad, m, v, delta)
        _f32(grad, m, v, delta)
        D = adam_delta_bound(t, lr, beta1, beta2)
        if D is None:
            raise ValueError("run_adam: no Adam delta bound for beta1^2 >= beta2 (use adam + run)")
        s = adam_scalars(t, lr, beta1, beta2, eps, grad_scale)
        vers = tuple(f._version for f in self._factor_reps)
        if self._factor_versions is not None and vers != self._factor_versions:
            # the factors changed in place since the constant panel halves / maxima were packed
            check(self._lib.hdp_delta_plan_invalidate(self._h), "hdp_delta_plan_invalidate")
        self._factor_versions = vers
        check(self._lib.hdp_delta_plan_run_adam(self._h, grad.data_ptr(), m.data_ptr(), v.data_ptr(), delta.data_ptr(),
                                                *s, D, int(bool(zero_grad)), _stream()), "hdp_delta_plan_run_adam")

    def fused_fallback(self) -> bool:
        """Whether the last run_adam re-packed from the live deltas (a delta above the bound; synchronises)."""
        import ctypes
        x = ctypes.c_int()
        check(self._lib.hdp_delta_plan_fused_fallback(self._h, ctypes.byref(x)), "hdp_delta_plan_fused_fallback")
        return bool(x.value)

    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.hdp_delta_plan_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def adam_delta_bound(t: int, lr: float, beta1: float, beta2: float) -> Optional[float]:
    """Upper bound of |delta| = |lr m_hat / (sqrt(v_hat) + eps)| after step t of hp:356-373 from zero
    moments: by Cauchy-Schwarz over the moment sums, |m_t| <= sqrt(v_t) (1 - b1) / sqrt(1 - b2) *
    sqrt(sum_j<t rho^j), rho = b1^2 / b2, so |m_hat| / sqrt(v_hat) <= that factor * sqrt(1 - b2^t) /
    (1 - b1^t) (<= 7.27 for 0.9 / 0.999; 1 at t = 1).  A 1 % margin covers the float32 rounding of the
    kernel's op sequence.  None where the series diverges (b1^2 >= b2)."""
    rho = beta1 * beta1 / beta2
    if not (0.0 <= rho < 1.0) or not (0.0 <= beta1 < 1.0) or not (0.0 < beta2 < 1.0) or t < 1:
        return None
    c = (1 - beta1) / math.sqrt(1 - beta2) * math.sqrt((1 - rho ** t) / (1 - rho)) * math.sqrt(1 - beta2 ** t) / (1 - beta1 ** t)
    return abs(lr) * c * 1.01


def adam_scalars(t: int, lr: float, beta1: float, beta2: float, eps: float, grad_scale: float = 1e16):
    """float32 scalars of hp:356-373 as torch evaluates them: Python floats (float64)
    combined first (1 - beta1, 1 - beta1 ** t, ...), then rounded to float32 when they
    meet a float32 tensor."""
    if t <= 0:
        raise ValueError("Adam step counter t must be >= 1 (t is incremented before the update, hp:350)")
    return (grad_scale, beta1, 1 - beta1, beta2, 1 - beta2, 1 - beta1 ** t, 1 - beta2 ** t, lr, eps)


_default: Optional[HipOps] = None


def default_ops() -> HipOps:
    global _default
    if _default is None:
        _default = HipOps()
    return _default
