"""Full-shape parity for every BASELINE.json configuration (SURVEY 8 shorthand P / M / L7 / Mi / L13).

For each configuration's distinct module shapes (out x in), at its own r and model dtype:

* K1 (SVD slice, hp:96-129) at the configuration's world size and at Wn = 8:
  - matrices with a KNOWN spectrum (W = Q1 diag(s) Q2^T, s a power law, built in float64):
    singular values vs s within 1e-4 relative (which also proves they are the TOP k), and the
    size-independent properties of every returned triplet -- ||W v_i - s_i u_i|| / s_i and
    ||W^T u_i - s_i v_i|| / s_i <= 1e-4, U_k and V_k orthonormal to 1e-4 -- so the check does not
    depend on how well separated neighbouring singular values are;
  - the bench's own initialisation (Gaussian N(0, 0.02^2), a near-flat Marchenko-Pastur
    spectrum) for the LLaMA-2-7B shapes: singular values vs numpy's float64 SVD, same
    properties (vectors compared up to sign would be ill-posed at these gaps).
* K2 (probe backward, hp:139 + autograd) at T = 700 rows (batch 2 x a ~350-token sample, the
  bench's mean padded micro-batch) for every distinct shape, model dtype inputs, vs the float64
  oracle, 1e-5 relative.
* K3 + K4 (Adam + the grouped delta-GEMM merge, hp:356-394): one plan holding one module of
  every distinct shape, at Wn = 1 (f32 MFMA) and Wn = 8 (K = 2 r 8, bf16x3 MFMA; bf16 models
  with the reference's per-rank bf16 rounding of the running dW).  f32: merged update vs the
  float64 truth 1e-5; bf16: vs the reference loop (oracle delta_w in bf16) within the bf16 bar,
  with the update itself checked (not only W) and the fraction of differing elements bounded.

Configurations (BASELINE.json `configs`): P = Qwen2.5-0.5B r16 fp32 (world size 2), M = the 4096^2
q_proj microbench, L7 = LLaMA-2-7B r16 fp32, Mi = Mistral-7B r64 bf16, L13 = LLaMA-2-13B r128 bf16.
"""
import numpy as np
import pytest
import torch

from oracle import hdpissa_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"

# config -> (dtype, r, configured world size, distinct module shapes (out, in) with their names)
CONFIGS = {
    "qwen2.5-0.5b": ("float32", 16, 2, {"q_proj": (896, 896), "k_proj": (128, 896), "gate_proj": (4864, 896),
                                        "down_proj": (896, 4864)}),
    "qproj-microbench": ("float32", 16, 8, {"q_proj": (4096, 4096)}),
    "llama2-7b": ("float32", 16, 8, {"q_proj": (4096, 4096), "gate_proj": (11008, 4096),
                                     "down_proj": (4096, 11008)}),
    "mistral-7b": ("bfloat16", 64, 8, {"q_proj": (4096, 4096), "k_proj": (1024, 4096), "gate_proj": (14336, 4096),
                                       "down_proj": (4096, 14336)}),
    "llama2-13b": ("bfloat16", 128, 8, {"q_proj": (5120, 5120), "gate_proj": (13824, 5120),
                                        "down_proj": (5120, 13824)}),
}
SHAPE_CASES = [(cfg, name) for cfg, (_, _, _, shapes) in CONFIGS.items() for name in shapes]


@pytest.fixture(scope="module")
def ops():
    from hdpissa_amd.ops import default_ops
    return default_ops()


def _t(a, dtype=torch.float32):
    return torch.as_tensor(np.ascontiguousarray(a)).to(DEV).to(dtype)


def _np(t):
    return t.detach().float().cpu().numpy()


def _tdt(dt):
    return torch.bfloat16 if dt == "bfloat16" else torch.float32


# ----------------------------------------------------------------------------------- K1
def _known_spectrum(out, inn, seed):
    """W = Q1 diag(s) Q2^T with Haar-like orthonormal Q1 (out x k0), Q2 (in x k0) and a power-law
    spectrum s_i = 0.5 (i + 1)^-0.35 (a pretrained weight's shape, every gap >= 3e-4 relative at
    i < 1024).  Built in float64 on the device (a construction of the input, not the checker);
    returns the float32 matrix (host) and s."""
    k0 = min(out, inn)
    gen = torch.Generator(device=DEV)
    gen.manual_seed(seed)
    q1, _ = torch.linalg.qr(torch.randn(out, k0, dtype=torch.float64, device=DEV, generator=gen))
    q2, _ = torch.linalg.qr(torch.randn(inn, k0, dtype=torch.float64, device=DEV, generator=gen))
    s = 0.5 * (torch.arange(k0, dtype=torch.float64, device=DEV) + 1.0) ** -0.35
    W = ((q1 * s) @ q2.T).float()
    return W.cpu().numpy(), s.cpu().numpy()


def _triplet_checks(W, A_all, B_all, S, r, wn, tol=1e-4):
    """Size-independent checks of the returned triplets (float64, host).  Our factors are
    A_d = diag(sqrt s_d) V_d^T and B_d = U_d diag(sqrt s_d) (hp:122-125)."""
    k = r * wn
    sq = np.sqrt(S[:k])
    V = (A_all[:k].astype(np.float64) / sq[:, None]).T                   # in x k
    U = np.concatenate([B_all[d].astype(np.float64) for d in range(wn)], axis=1) / sq[None, :]  # out x k
    W64 = W.astype(np.float64)
    res_v = np.linalg.norm(W64 @ V - U * S[None, :k], axis=0) / S[:k]
    res_u = np.linalg.norm(W64.T @ U - V * S[None, :k], axis=0) / S[:k]
    assert res_v.max() < tol, ("||W v - s u|| / s", float(res_v.max()), int(res_v.argmax()))
    assert res_u.max() < tol, ("||W^T u - s v|| / s", float(res_u.max()), int(res_u.argmax()))
    eye = np.eye(k)
    assert np.abs(V.T @ V - eye).max() < tol, "V_k not orthonormal"
    assert np.abs(U.T @ U - eye).max() < tol, "U_k not orthonormal"
    # the factor norms carry sqrt(s) exactly as the reference's diag products do
    s_got = np.linalg.norm(A_all[:k].astype(np.float64), axis=1) * \
        np.concatenate([np.linalg.norm(B_all[d].astype(np.float64), axis=0) for d in range(wn)])
    assert np.allclose(s_got, S[:k], rtol=tol)


@pytest.mark.parametrize("cfg,name", SHAPE_CASES)
def test_config_svd_known_spectrum(ops, cfg, name):
    dt, r, wn_cfg, shapes = CONFIGS[cfg]
    out, inn = shapes[name]
    W, s = _known_spectrum(out, inn, seed=out * 31 + inn)
    if dt == "bfloat16":
        # the model weight is bf16: its spectrum moves by ~4e-3 relative, so the reference
        # values are the float64 singular values of the rounded matrix (numpy: the SVD below
        # 4096, the eigenvalues of the float64 Gram matrix above -- exact for the top k)
        W = O.round_bf16(W)
        W64 = W.astype(np.float64)
        if max(out, inn) <= 4096:
            s = np.linalg.svd(W64, compute_uv=False)
        else:
            gram = W64.T @ W64 if inn <= out else W64 @ W64.T
            s = np.sqrt(np.maximum(np.linalg.eigvalsh(gram)[::-1], 0.0))
            del gram
        del W64
    for wn in sorted({1, wn_cfg, 8}):  # (wn = 1: k = r; k <= 32 at n >= 2048 takes the block-Krylov solve, r05)
        k = r * wn
        if k > min(out, inn):
            continue
        A_all, B_all, S = ops.svd_topk(_t(W, _tdt(dt)), r, wn)
        torch.cuda.synchronize()
        A_all, B_all, S = _np(A_all), _np(B_all), S.cpu().numpy()
        assert np.all(np.diff(S) <= 0), "singular values must come back descending"
        assert np.allclose(S, s[:k], rtol=1e-4), (cfg, name, wn, float(np.max(np.abs(S / s[:k] - 1))))
        _triplet_checks(W, A_all, B_all, S, r, wn)


@pytest.mark.parametrize("out,inn", [(4096, 4096), (11008, 4096)])
def test_config_svd_gaussian_bench_init(ops, out, inn):
    """The bench's random init (N(0, 0.02^2), LLaMA-2-7B shapes) at Wn = 8, r = 16: near-flat
    spectrum at the Marchenko-Pastur edge -- singular values vs numpy float64, triplet properties."""
    g = np.random.default_rng(out + inn)
    W = (g.standard_normal((out, inn)) * 0.02).astype(np.float32)
    r, wn = 16, 8
    A_all, B_all, S = ops.svd_topk(_t(W), r, wn)
    torch.cuda.synchronize()
    A_all, B_all, S = _np(A_all), _np(B_all), S.cpu().numpy()
    s_ref = np.linalg.svd(W.astype(np.float64), compute_uv=False)[:r * wn]
    assert np.allclose(S, s_ref, rtol=1e-4), float(np.max(np.abs(S / s_ref - 1)))
    _triplet_checks(W, A_all, B_all, S, r, wn)


@pytest.mark.parametrize("out,inn", [(4096, 4096), (11008, 4096), (4096, 11008)])
def test_config_svd_truncated_bench_init(ops, monkeypatch, capfd, out, inn):
    """r05, north_star (1)'s truncated SVD: k = r Wn <= 64 at n >= 2048 runs block Krylov on the Gram
    (Rayleigh-Ritz over 1024 directions, 2048 for k > 32, explicit residual check, full dsyevd only as the
    fallback).  The
    bench's own Gaussian init is the hardest case for it (near-flat Marchenko-Pastur edge): at k = 16 the
    truncated solve must be ACCEPTED (HDP_EIG_TRACE) and meet the same bars as the full solve -- singular
    values vs numpy float64 1e-4, triplet residuals and orthonormality 1e-4; k = 32 is checked either way
    (it may fall back).  Also the batched entry (three matrices of one n in one call)."""
    monkeypatch.setenv("HDP_EIG_TRACE", "1")
    g = np.random.default_rng(out * 3 + inn)
    W = (g.standard_normal((out, inn)) * 0.02).astype(np.float32)
    s_ref = np.linalg.svd(W.astype(np.float64), compute_uv=False)
    for r, wn in ((16, 1), (16, 2)):
        capfd.readouterr()
        A_all, B_all, S = ops.svd_topk(_t(W), r, wn)
        torch.cuda.synchronize()
        err = capfd.readouterr().err
        if r * wn == 16:
            assert "block Krylov" in err and "accepted" in err, err
        A_all, B_all, S = _np(A_all), _np(B_all), S.cpu().numpy()
        assert np.allclose(S, s_ref[:r * wn], rtol=1e-4), float(np.max(np.abs(S / s_ref[:r * wn] - 1)))
        _triplet_checks(W, A_all, B_all, S, r, wn)
    if (out, inn) != (4096, 11008):  # k = 64 (Mistral-7B r64 at Wn = 1): m = 2048, must be accepted too
        capfd.readouterr()
        A_all, B_all, S = ops.svd_topk(_t(W), 64, 1)
        torch.cuda.synchronize()
        err = capfd.readouterr().err
        assert "block Krylov" in err and "m=2048" in err and "accepted" in err, err
        A_all, B_all, S = _np(A_all), _np(B_all), S.cpu().numpy()
        assert np.allclose(S, s_ref[:64], rtol=1e-4), float(np.max(np.abs(S / s_ref[:64] - 1)))
        _triplet_checks(W, A_all, B_all, S, 64, 1)
    if (out, inn) == (4096, 4096):
        Ws = [W] + [(g.standard_normal((out, inn)) * 0.02).astype(np.float32) for _ in range(2)]
        capfd.readouterr()
        res = ops.svd_topk_batch([_t(x) for x in Ws], 16, 1)
        torch.cuda.synchronize()
        assert "accepted" in capfd.readouterr().err
        for x, (A_all, B_all, S) in zip(Ws, res):
            s2 = np.linalg.svd(x.astype(np.float64), compute_uv=False)[:16]
            S = S.cpu().numpy()
            assert np.allclose(S, s2, rtol=1e-4)
            _triplet_checks(x, _np(A_all), _np(B_all), S, 16, 1)


def test_config_svd_truncated_k128(ops, capfd, monkeypatch):
    """k = 128 (LLaMA-2-13B r128 at Wn = 1) at n = 5120: block Krylov over 3072 directions, accepted at the bench's
    Gaussian init and held to the full solve's bars (singular values vs numpy float64, triplet residuals and
    orthonormality 1e-4)."""
    monkeypatch.setenv("HDP_EIG_TRACE", "1")
    g = np.random.default_rng(5120)
    W = (g.standard_normal((5120, 5120)) * 0.02).astype(np.float32)
    s_ref = np.linalg.svd(W.astype(np.float64), compute_uv=False)
    capfd.readouterr()
    A_all, B_all, S = ops.svd_topk(_t(W), 128, 1)
    torch.cuda.synchronize()
    err = capfd.readouterr().err
    assert "block Krylov" in err and "m=3072" in err and "accepted" in err, err
    A_all, B_all, S = _np(A_all), _np(B_all), S.cpu().numpy()
    assert np.allclose(S, s_ref[:128], rtol=1e-4), float(np.max(np.abs(S / s_ref[:128] - 1)))
    _triplet_checks(W, A_all, B_all, S, 128, 1)


@pytest.mark.parametrize("out,inn", [(4096, 4096), (11008, 4096)])
def test_config_svd_truncated_k128_n4096(ops, capfd, monkeypatch, out, inn):
    """k = 128 at n = 4096 -- LLaMA-2-7B r16 at Wn = 8, the 8-GPU headline's init (VERDICT r05 missing #3): block
    Krylov over 3072 directions, accepted at the bench's Gaussian init and held to the full solve's bars (singular
    values vs numpy float64, triplet residuals and orthonormality 1e-4), single and batched (the sharded init's
    per-rank batch of one n)."""
    monkeypatch.setenv("HDP_EIG_TRACE", "1")
    g = np.random.default_rng(out + 7 * inn)
    W = (g.standard_normal((out, inn)) * 0.02).astype(np.float32)
    s_ref = np.linalg.svd(W.astype(np.float64), compute_uv=False)
    capfd.readouterr()
    A_all, B_all, S = ops.svd_topk(_t(W), 16, 8)
    torch.cuda.synchronize()
    err = capfd.readouterr().err
    assert "block Krylov" in err and "k=128" in err and "m=3072" in err and "accepted" in err, err
    A_all, B_all, S = _np(A_all), _np(B_all), S.cpu().numpy()
    assert np.allclose(S, s_ref[:128], rtol=1e-4), float(np.max(np.abs(S / s_ref[:128] - 1)))
    _triplet_checks(W, A_all, B_all, S, 16, 8)
    if (out, inn) == (4096, 4096):
        W2 = (g.standard_normal((out, inn)) * 0.02).astype(np.float32)
        capfd.readouterr()
        res = ops.svd_topk_batch([_t(W), _t(W2)], 16, 8)
        torch.cuda.synchronize()
        assert "accepted" in capfd.readouterr().err
        for x, (A2, B2, S2) in zip((W, W2), res):
            s2 = np.linalg.svd(x.astype(np.float64), compute_uv=False)[:128]
            S2 = S2.cpu().numpy()
            assert np.allclose(S2, s2, rtol=1e-4)
            _triplet_checks(x, _np(A2), _np(B2), S2, 16, 8)


@pytest.mark.parametrize("batch", [1, 3])
def test_config_svd_krylov_fallback(ops, capfd, monkeypatch, batch):
    """The truncated solve's fallback: a basis far too shallow for the bench's Gaussian init
    (HDP_KRY_M = 128 directions for k = 16) misses the 1e-5 Ritz residual bar, so the batch must drop to the
    full dsyevd on the Grams the Krylov pass left intact -- 'full solve' in HDP_EIG_TRACE, then the full solve's
    bars (singular values vs numpy float64, triplet residuals and orthonormality 1e-4) for every item, through
    the single-matrix and the batched entry."""
    monkeypatch.setenv("HDP_EIG_TRACE", "1")
    monkeypatch.setenv("HDP_KRY_M", "128")
    g = np.random.default_rng(2048 + batch)
    Ws = [(g.standard_normal((2048 + 512 * i, 2048)) * 0.02).astype(np.float32) for i in range(batch)]
    capfd.readouterr()
    if batch == 1:
        res = [ops.svd_topk(_t(Ws[0]), 16, 1)]
    else:
        res = ops.svd_topk_batch([_t(x) for x in Ws], 16, 1)
    torch.cuda.synchronize()
    err = capfd.readouterr().err
    assert "block Krylov" in err and "m=128" in err and "full solve" in err and "accepted" not in err, err
    for x, (A_all, B_all, S) in zip(Ws, res):
        s_ref = np.linalg.svd(x.astype(np.float64), compute_uv=False)[:16]
        S = S.cpu().numpy()
        assert np.allclose(S, s_ref, rtol=1e-4), float(np.max(np.abs(S / s_ref - 1)))
        _triplet_checks(x, _np(A_all), _np(B_all), S, 16, 1)


# ----------------------------------------------------------------------------------- K2
@pytest.mark.parametrize("cfg,name", SHAPE_CASES)
def test_config_probe_full_shape(ops, cfg, name):
    dt, r, _, shapes = CONFIGS[cfg]
    out, inn = shapes[name]
    T = 700
    g = np.random.default_rng(out + 3 * inn + r)
    X = g.standard_normal((T, inn)).astype(np.float32)
    G = (g.standard_normal((T, out)) * 1e-3).astype(np.float32)
    if dt == "bfloat16":
        X, G = O.round_bf16(X), O.round_bf16(G)
    A = (g.standard_normal((r, inn)) * 0.05).astype(np.float32)
    B = (g.standard_normal((out, r)) * 0.05).astype(np.float32)
    alpha = float(r)  # alpha = r -> alpha_eff 1 (bench configs)
    scale = float(np.float32(1.0) * np.float32(1e-16))
    gA0 = (g.standard_normal((r, inn)) * 1e-18).astype(np.float32)
    gB0 = (g.standard_normal((out, r)) * 1e-18).astype(np.float32)
    tgA, tgB = _t(gA0), _t(gB0)
    tX, tG = _t(X, _tdt(dt)), _t(G, _tdt(dt))
    ops.probe_grads(tX, tG, _t(A), _t(B), tgA, tgB, scale, True, Bt=_t(B).t().contiguous())
    torch.cuda.synchronize()
    rA, rB = O.probe_grads(X, G, A, B, O.alpha_eff(alpha, r))
    assert O.rel_err(_np(tgA), gA0 + rA) < 1e-5
    assert O.rel_err(_np(tgB), gB0 + rB) < 1e-5


# ----------------------------------------------------------------------------------- K3 + K4
def _layer_operands(g, shapes, r, wn, dt):
    """Per module: every rank's factors (SVD-scaled magnitudes), probe grads, Adam state; the
    arena-like flat buffers the step consumes (segment stride F per rank)."""
    mods = []
    for name, (out, inn) in shapes.items():
        A = [(g.standard_normal((r, inn)) * 0.1).astype(np.float32) for _ in range(wn)]
        B = [(g.standard_normal((out, r)) * 0.1).astype(np.float32) for _ in range(wn)]
        gA = [(g.standard_normal((r, inn)) * 1e-14).astype(np.float32) for _ in range(wn)]
        gB = [(g.standard_normal((out, r)) * 1e-14).astype(np.float32) for _ in range(wn)]
        W = (g.standard_normal((out, inn)) * 0.02).astype(np.float32)
        if dt == "bfloat16":
            W = O.round_bf16(W)
        mods.append(dict(name=name, out=out, inn=inn, A=A, B=B, gA=gA, gB=gB, W=W))
    offs, off = [], 0
    for m in mods:
        oa = off
        ob = oa + (m["inn"] * r + 63) // 64 * 64
        off = ob + (m["out"] * r + 63) // 64 * 64
        offs.append((oa, ob))
    F = off
    fac = np.zeros((wn, F), np.float32)
    grad = np.zeros((wn, F), np.float32)
    for m, (oa, ob) in zip(mods, offs):
        for i in range(wn):
            fac[i, oa:oa + r * m["inn"]] = m["A"][i].reshape(-1)
            fac[i, ob:ob + m["out"] * r] = m["B"][i].reshape(-1)
            grad[i, oa:oa + r * m["inn"]] = m["gA"][i].reshape(-1)
            grad[i, ob:ob + m["out"] * r] = m["gB"][i].reshape(-1)
    return mods, offs, F, fac, grad


@pytest.mark.parametrize("wn", [1, 8])
@pytest.mark.parametrize("cfg", list(CONFIGS))
def test_config_layer_step_plan(ops, cfg, wn):
    """Adam (K3) over the flat arena of every rank, then ONE grouped K4 plan over one module of
    each distinct shape: W_res += sum_i (B'_i A'_i - B_i A_i) in rank order (hp:356-394)."""
    from hdpissa_amd._lib import HDP_DW_MERGE
    dt, r, _, shapes = CONFIGS[cfg]
    if wn * r > min(min(s) for s in shapes.values()):
        shapes = {k: v for k, v in shapes.items() if wn * r <= min(v)}
    g = np.random.default_rng(wn * 100 + r)
    mods, offs, F, fac, grad = _layer_operands(g, shapes, r, wn, dt)
    t, lr = 3, 2e-3  # a large lr makes the update visible next to bf16 W
    m0 = (g.standard_normal((wn, F)) * 1e-2).astype(np.float32)
    v0 = np.abs(g.standard_normal((wn, F)) * 1e-4).astype(np.float32)
    tfac, tgrad, tm, tv = _t(fac), _t(grad), _t(m0), _t(v0)
    tdelta = torch.zeros(wn, F, device=DEV)
    for i in range(wn):
        ops.adam(tgrad[i], tm[i], tv[i], tdelta[i], t, lr, 0.9, 0.999, 1e-8, zero_grad=True)
    torch.cuda.synchronize()
    # K3 bit-exactness at full arena size (rank 0; every rank runs the same kernel)
    m_ref, v_ref, d_ref = O.adam_factors(grad[0], m0[0], v0[0], t, lr)
    assert np.array_equal(_np(tm[0]), m_ref) and np.array_equal(_np(tv[0]), v_ref)
    delta = _np(tdelta)
    assert np.max(np.abs(delta[0] - d_ref) / (np.abs(d_ref) + 1e-30)) < 2.5e-7
    assert not torch.any(tgrad)
    # K4: one plan, every module, K = 2 r wn
    tdt = _tdt(dt)
    Ws = [_t(m["W"], tdt) for m in mods]
    fd, ff = tdelta.view(-1), tfac.view(-1)
    items = [(m["out"], m["inn"], r, wn, fd[oa:], fd[ob:], F, ff[oa:], ff[ob:], F, Wt)
             for m, (oa, ob), Wt in zip(mods, offs, Ws)]
    plan = ops.delta_plan(items, HDP_DW_MERGE, dt == "bfloat16")
    plan.run()
    torch.cuda.synchronize()
    plan.close()
    for m, (oa, ob), Wt in zip(mods, offs, Ws):
        dA = [delta[i, oa:oa + r * m["inn"]].reshape(r, m["inn"]) for i in range(wn)]
        dB = [delta[i, ob:ob + m["out"] * r].reshape(m["out"], r) for i in range(wn)]
        got = _np(Wt)
        if dt == "float32":
            upd = O.delta_w_exact(dA, dB, m["A"], m["B"])
            assert O.rel_err(got - m["W"], upd) < 1e-5, (cfg, m["name"], wn)
        else:
            dW = O.delta_w(dA, dB, m["A"], m["B"], dt)
            ref = O.merge(m["W"], dW, dt)
            assert O.rel_err(got, ref) < 2e-2, (cfg, m["name"], wn)
            # the update itself, not only W: bf16-level agreement, and the reference's
            # rank-ordered bf16 rounding reproduced for nearly every element
            assert O.rel_err(got - m["W"], ref - m["W"]) < 2e-2, (cfg, m["name"], wn)
            assert np.mean(got != ref) < 0.02, (cfg, m["name"], wn, float(np.mean(got != ref)))
