"""CPU oracle for the HD-PiSSA per-step distributed orthogonal-adapter update.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module, and only as the
checker / reported CPU baseline -- never as the thing measured or shipped.  The
product path (``hd-pissa_amd/hdpissa_amd``) never imports it and fails loudly
when its HIP library is missing.

This is a from-scratch numpy restatement of the arithmetic in the reference
``/root/reference/hd_pissa.py`` (abbreviated ``hp:``).  Every function cites
the lines it follows.  Parity of this oracle is *pinned* by golden vectors
captured from the reference itself (``tests/golden/make_golden.py`` imports
``hd_pissa`` in the build container and runs its own ``CustomLinearLayer``,
autograd and the literal optimizer-step block ``hp:352-398`` under gloo);
``tests/test_oracle_golden.py`` checks every function below against them.

Dtype conventions mirror the reference: factors A, B, grads, Adam moments and
the per-step delta are float32; ``W_res`` is the model dtype (float32 or
bfloat16).  numpy has no bfloat16, so bf16 tensors are carried as float32
arrays whose values are exactly bf16-representable (``round_bf16``).
"""
from __future__ import annotations

import math
from typing import List, Sequence, Tuple

import numpy as np

F32 = np.float32


# ----------------------------------------------------------------------------
# bf16 helpers (torch's float32 -> bfloat16 cast is round-to-nearest-even)
# ----------------------------------------------------------------------------
def round_bf16(x: np.ndarray) -> np.ndarray:
    """Round float32 values to the nearest bf16 value (RNE), returned as float32."""
    x = np.ascontiguousarray(x, dtype=F32)
    u = x.view(np.uint32).astype(np.uint64)
    bias = ((u >> 16) & 1) + 0x7FFF
    r = ((u + bias) >> 16) << 16
    out = r.astype(np.uint32).view(F32)
    nan = np.isnan(x)
    if nan.any():
        out = out.copy()
        out[nan] = np.nan
    return out


# ----------------------------------------------------------------------------
# C1: SVD-slice initializer  (hp:96-134)
# ----------------------------------------------------------------------------
def alpha_eff(alpha: float, ranks_per_gpu: int) -> float:
    """``self.alpha = alpha // ranks_per_gpu`` -- Python floor division (hp:103)."""
    return alpha // ranks_per_gpu


def svd_full(W: np.ndarray) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """``U, S, V = torch.svd(W.float())`` (hp:106-109), computed in float64.

    Returns U (out x k), S (k,), V (in x k) with k = min(out, in), descending S.
    The reference runs the SVD in float32; float64 here is the exact SVD of the
    float32 matrix, so it is the better yardstick for both implementations.
    """
    W64 = np.asarray(W, dtype=F32).astype(np.float64)
    U, S, Vh = np.linalg.svd(W64, full_matrices=False)
    return U, S, Vh.T


def svd_slice(W: np.ndarray, device_id: int, world_size: int, ranks_per_gpu: int,
              model_dtype: str = "float32"):
    """Rank ``device_id``'s factors (hp:111-129).

    A = diag(sqrt(S[d*r:(d+1)*r])) @ V[:, slice]^T   (r x in, float32)   hp:122-124
    B = U[:, slice] @ diag(sqrt(S[slice]))           (out x r, float32)  hp:125
    W_res = W in the model dtype -- NOT W - B A                            hp:129
    Returns (A, B, W_res, S_sub).
    """
    U, S, V = svd_full(W)
    start = device_id * ranks_per_gpu                     # hp:116
    end = (device_id + 1) * ranks_per_gpu                 # hp:117
    S_sub = S[start:end]                                  # hp:119
    sq = np.sqrt(S_sub)                                   # hp:122
    A = (sq[:, None] * V[:, start:end].T).astype(F32)     # hp:124
    B = (U[:, start:end] * sq[None, :]).astype(F32)       # hp:125
    W32 = np.asarray(W, dtype=F32)
    W_res = round_bf16(W32) if model_dtype == "bfloat16" else W32.copy()
    return A, B, W_res, S_sub


def align_signs(X: np.ndarray, Y: np.ndarray, axis: int) -> np.ndarray:
    """Flip the sign of each row (axis=1 -> rows are vectors) or column (axis=0)
    of X so it best matches Y: SVD vectors are defined up to sign per triplet."""
    if axis == 1:  # rows are the singular vectors (A: r x in)
        s = np.sign(np.sum(X.astype(np.float64) * Y, axis=1))
        s[s == 0] = 1
        return X * s[:, None]
    s = np.sign(np.sum(X.astype(np.float64) * Y, axis=0))
    s[s == 0] = 1
    return X * s[None, :]


# ----------------------------------------------------------------------------
# C2: adapter probe forward/backward  (hp:136-140 + autograd)
# ----------------------------------------------------------------------------
def probe_forward(x: np.ndarray, W_res: np.ndarray, bias=None) -> np.ndarray:
    """Base linear ``F.linear(x, W_res, bias)`` (hp:139).  The adapter term is
    scaled by 1e-16 and vanishes in rounding; the golden vectors confirm the
    reference output equals the base linear on the fixture inputs."""
    y = np.asarray(x, np.float64) @ np.asarray(W_res, np.float64).T
    if bias is not None:
        y = y + np.asarray(bias, np.float64)
    return y


def probe_grads(x: np.ndarray, G: np.ndarray, A: np.ndarray, B: np.ndarray,
                alpha: float) -> Tuple[np.ndarray, np.ndarray]:
    """Gradients autograd leaves in ``A.grad`` / ``B.grad`` (hp:139).

    M = (B @ A) * 1e-16 * alpha; out = x32 @ M^T  =>  dM = G32^T x32,
    dB = (1e-16 alpha) dM A^T,  dA = (1e-16 alpha) B^T dM.
    Computed in float64 (the reference's float32 rounding is within 1e-6).
    x: (..., in), G: (..., out) -- any leading dims (batch, seq).
    """
    X = np.asarray(x, np.float64).reshape(-1, np.shape(x)[-1])
    Gm = np.asarray(G, np.float64).reshape(-1, np.shape(G)[-1])
    s = float(np.float32(1e-16)) * float(np.float32(alpha))
    H = X @ np.asarray(A, np.float64).T        # T x r
    J = Gm @ np.asarray(B, np.float64)          # T x r
    gA = s * (J.T @ X)                          # r x in
    gB = s * (Gm.T @ H)                         # out x r
    return gA, gB


def probe_dense_reference(x: np.ndarray, G: np.ndarray, A: np.ndarray, B: np.ndarray, alpha: float,
                          W_res: np.ndarray):
    """The reference's own per-micro-step arithmetic for one layer, float32, literally:
    forward  y = x W_res^T + x32 (1e-16 alpha B A)^T      (hp:139, M materialised out x in)
    backward dX = G W_res + G M,  dM = G^T x32,  dB = s dM A^T,  dA = s B^T dM   (autograd)
    Used as the CPU-baseline workload (its cost is what the reference pays); returns (y, dX, dA, dB)."""
    X = np.asarray(x, F32).reshape(-1, np.shape(x)[-1])
    Gm = np.asarray(G, F32).reshape(-1, np.shape(G)[-1])
    M = (np.asarray(B, F32) @ np.asarray(A, F32)) * F32(1e-16) * F32(alpha)
    y = X @ np.asarray(W_res, F32).T + X @ M.T
    dX = Gm @ np.asarray(W_res, F32) + Gm @ M
    dM = (Gm.T @ X) * F32(alpha) * F32(1e-16)
    return y, dX, np.asarray(B, F32).T @ dM, dM @ np.asarray(A, F32).T


def probe_dense_adapter_only(x: np.ndarray, G: np.ndarray, A: np.ndarray, B: np.ndarray, alpha: float):
    """The adapter-term share of ``probe_dense_reference`` (what hp:139 adds on top of the
    base linear): M = 1e-16 alpha B A; y_ad = x M^T; dX_ad = G M; dM = G^T x; dA, dB.
    float32, the reference's evaluation order.  Returns (dA, dB)."""
    X = np.asarray(x, F32).reshape(-1, np.shape(x)[-1])
    Gm = np.asarray(G, F32).reshape(-1, np.shape(G)[-1])
    M = (np.asarray(B, F32) @ np.asarray(A, F32)) * F32(1e-16) * F32(alpha)
    _y_ad = X @ M.T
    _dx_ad = Gm @ M
    dM = (Gm.T @ X) * F32(alpha) * F32(1e-16)
    return np.asarray(B, F32).T @ dM, dM @ np.asarray(A, F32).T


# ----------------------------------------------------------------------------
# C4: Adam on factors  (hp:297-300, 356-373)
# ----------------------------------------------------------------------------
def adam_factors(grad_raw: np.ndarray, m: np.ndarray, v: np.ndarray, t: int, lr: float,
                 beta1: float = 0.9, beta2: float = 0.999, eps: float = 1e-8):
    """One Adam update on a factor, float32 semantics of the reference.

    grad = raw_grad * 1e16                    hp:356-357
    m = beta1 m + (1-beta1) grad              hp:360/363
    v = beta2 v + (1-beta2) grad^2            hp:361/364
    m_hat = m / (1-beta1^t); v_hat likewise   hp:366-369  (t already incremented, hp:350)
    delta = lr m_hat / (sqrt(v_hat) + eps)    hp:372-373
    Returns (m_new, v_new, delta) as float32.
    """
    g = np.asarray(grad_raw, F32) * F32(1e16)
    m_new = F32(beta1) * np.asarray(m, F32) + F32(1 - beta1) * g
    v_new = F32(beta2) * np.asarray(v, F32) + F32(1 - beta2) * (g * g)
    m_hat = m_new / F32(1 - beta1 ** t)
    v_hat = v_new / F32(1 - beta2 ** t)
    delta = F32(lr) * m_hat / (np.sqrt(v_hat) + F32(eps))
    return m_new.astype(F32), v_new.astype(F32), delta.astype(F32)


# ----------------------------------------------------------------------------
# C6: Delta-W formation  (hp:389-392) and C7 merge (hp:394)
# ----------------------------------------------------------------------------
def delta_w(dA_list: Sequence[np.ndarray], dB_list: Sequence[np.ndarray],
            A_list: Sequence[np.ndarray], B_list: Sequence[np.ndarray],
            model_dtype: str = "float32") -> np.ndarray:
    """The reference loop, ranks summed in order i = 0..Wn-1 (hp:389-392):

        dW = zeros_like(W_res);  for i: dW -= dB_i @ A_i + B_i @ dA_i - dB_i @ dA_i

    The bracket is float32 (factors are float32).  ``zeros_like(W_res)`` has the
    *model* dtype, so for a bf16 model the running sum is rounded to bf16 after
    every rank's term (torch computes ``bf16 -= f32`` in float32, then casts).
    """
    out, inn = dB_list[0].shape[0], A_list[0].shape[1]
    dW = np.zeros((out, inn), F32)
    for dA, dB, A, B in zip(dA_list, dB_list, A_list, B_list):
        dA, dB, A, B = (np.asarray(z, F32) for z in (dA, dB, A, B))
        dW = dW - (dB @ A + B @ dA - dB @ dA)
        if model_dtype == "bfloat16":
            dW = round_bf16(dW)
    return dW


def delta_w_exact(dA_list, dB_list, A_list, B_list) -> np.ndarray:
    """Same quantity as ``delta_w`` in float64: sum_i (B'_i A'_i - B_i A_i) with
    A' = A - dA, B' = B - dB.  Used as the tight-tolerance yardstick."""
    acc = None
    for dA, dB, A, B in zip(dA_list, dB_list, A_list, B_list):
        dA, dB, A, B = (np.asarray(z, np.float64) for z in (dA, dB, A, B))
        term = -(dB @ (A - dA) + B @ dA)
        acc = term if acc is None else acc + term
    return acc


def merge(W_res: np.ndarray, dW: np.ndarray, model_dtype: str = "float32") -> np.ndarray:
    """``W_res.data += delta_W_res.to(W_res.dtype)`` (hp:394).

    float32: W + dW.  bfloat16: dW is already bf16 (see ``delta_w``) and the
    in-place bf16 add rounds once: bf16(W + dW)."""
    W = np.asarray(W_res, F32)
    d = np.asarray(dW, F32)
    if model_dtype == "bfloat16":
        return round_bf16(W + round_bf16(d))
    return W + d


def pissa_residual(W: np.ndarray, A_list: Sequence[np.ndarray], B_list: Sequence[np.ndarray]) -> np.ndarray:
    """Opt-in PiSSA-residual storage (NOT the reference's default: hp:129 keeps W_res = W; the
    north star's "W_res formed by an MFMA GEMM"): W - sum_i B_i A_i over every rank's slice, in
    float64.  The effective weight W_res + sum_i B_i A_i equals W."""
    acc = np.asarray(W, np.float64).copy()
    for A, B in zip(A_list, B_list):
        acc -= np.asarray(B, np.float64) @ np.asarray(A, np.float64)
    return acc


# ----------------------------------------------------------------------------
# C9: learning-rate schedule  (hp:302-307, 338-344)
# ----------------------------------------------------------------------------
def total_steps(num_epochs: int, len_dataloader: int, accumulation_steps: int) -> int:
    """``num_epochs * len(dataloader) // accumulation_steps`` (hp:305)."""
    return num_epochs * len_dataloader // accumulation_steps


def warmup_from_ratio(warmup_steps: int, warmup_ratio: float, total: int) -> int:
    """hp:306-307."""
    if warmup_steps == 0 and warmup_ratio > 0:
        return int(warmup_ratio * total)
    return warmup_steps


def lr_at(t: int, initial_lr: float, warmup_steps: int, total: int, schedule: str) -> float:
    """Learning rate used at optimizer step with counter ``t`` (before ``t += 1``),
    hp:338-344."""
    if t < warmup_steps:
        return initial_lr * t / warmup_steps
    if schedule == "cosine":
        return 0.5 * initial_lr * (1 + math.cos(math.pi * (t - warmup_steps) / (total - warmup_steps)))
    return initial_lr * (1 - (t - warmup_steps) / (total - warmup_steps))


# ----------------------------------------------------------------------------
# Composition: one rank's view of the optimizer step for one module (hp:352-398)
# ----------------------------------------------------------------------------
def step_module(grads_A: List[np.ndarray], grads_B: List[np.ndarray],
                m_A: List[np.ndarray], v_A: List[np.ndarray],
                m_B: List[np.ndarray], v_B: List[np.ndarray],
                A_list: List[np.ndarray], B_list: List[np.ndarray],
                W_res: np.ndarray, t: int, lr: float, model_dtype: str = "float32",
                beta1: float = 0.9, beta2: float = 0.999, eps: float = 1e-8):
    """All ranks' data for one module -> (new W_res, per-rank (mA, vA, mB, vB), dW).

    ``t`` is the value after the increment at hp:350.  Every rank computes the
    same dW from the all-gathered factors (hp:379-392)."""
    dA_l, dB_l, states = [], [], []
    for i in range(len(A_list)):
        mA, vA, dA = adam_factors(grads_A[i], m_A[i], v_A[i], t, lr, beta1, beta2, eps)
        mB, vB, dB = adam_factors(grads_B[i], m_B[i], v_B[i], t, lr, beta1, beta2, eps)
        dA_l.append(dA)
        dB_l.append(dB)
        states.append((mA, vA, mB, vB))
    dW = delta_w(dA_l, dB_l, A_list, B_list, model_dtype)
    return merge(W_res, dW, model_dtype), states, dW


def rel_err(x, ref) -> float:
    """Norm-wise relative error ||x - ref|| / ||ref||."""
    x = np.asarray(x, np.float64)
    ref = np.asarray(ref, np.float64)
    den = np.linalg.norm(ref)
    return float(np.linalg.norm(x - ref) / (den if den > 0 else 1.0))
