"""Pin the CPU oracle to golden vectors captured from the reference itself.

Each test loads a fixture written by ``tests/golden/make_golden.py`` (which ran the
reference's own ``CustomLinearLayer``, autograd and the literal ``hp:352-398``
update block under gloo) and checks the oracle restatement against it.
"""
import glob
import os

import numpy as np
import pytest

from oracle import hdpissa_oracle as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    return np.load(os.path.join(GOLDEN, name))


def test_round_bf16_matches_torch():
    import torch
    x = torch.randn(10000) * torch.logspace(-30, 30, 10000)
    ref = x.to(torch.bfloat16).float().numpy()
    assert np.array_equal(O.round_bf16(x.numpy()), ref)


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "svd_*.npz"))))
def test_svd_slice(path):
    z = np.load(path)
    W = z["W"]
    dt = "bfloat16" if path.endswith("_bf16.npz") else "float32"
    U, S, V = O.svd_full(W)
    assert O.rel_err(S, z["S"]) < 1e-12
    for key in z.files:
        if not key.startswith("A_"):
            continue
        _, r, wn, d = key.split("_")
        r, wn, d = int(r[1:]), int(wn[1:]), int(d[1:])
        A, B, W_res, S_sub = O.svd_slice(W, d, wn, r, dt)
        Ar, Br = z[key], z[key.replace("A_", "B_")]
        # singular values: ||A_j|| * ||B_j|| = S_j
        s_ref = np.linalg.norm(Ar, axis=1) * np.linalg.norm(Br, axis=0)
        assert np.allclose(s_ref, S_sub, rtol=1e-4)
        # vectors up to per-triplet sign (hp:122-125)
        A_al = O.align_signs(A, Ar, axis=1)
        B_al = O.align_signs(B, Br, axis=0)
        assert O.rel_err(A_al, Ar) < 1e-4, key
        assert O.rel_err(B_al, Br) < 1e-4, key
        assert np.array_equal(W_res, W)  # W_res = W (hp:129)


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "probe_*.npz"))))
def test_probe_grads_accumulate(path):
    z = np.load(path)
    a_eff = O.alpha_eff(float(z["alpha"]), int(z["r"]))
    assert a_eff == float(z["alpha_eff"])
    bf16 = "bf16" in path
    gA = np.zeros_like(z["A"], dtype=np.float64)
    gB = np.zeros_like(z["B"], dtype=np.float64)
    for ms in range(3):
        # forward equals the base linear bit-for-bit on these inputs (hp:139)
        assert bool(z[f"y_equals_base{ms}"])
        y = O.probe_forward(z[f"x{ms}"], z["W"], z["bias"] if "bias" in z.files else None)
        assert O.rel_err(y, z[f"y{ms}"]) < (2e-2 if bf16 else 1e-5)
        dA, dB = O.probe_grads(z[f"x{ms}"], z[f"G{ms}"], z["A"], z["B"], a_eff)
        gA += dA
        gB += dB
        if a_eff == 0:
            assert not np.any(z[f"gA{ms}"]) and not np.any(z[f"gB{ms}"])
            continue
        assert O.rel_err(gA, z[f"gA{ms}"]) < 1e-5
        assert O.rel_err(gB, z[f"gB{ms}"]) < 1e-5


def test_lr_schedule():
    rows = _load("lr_schedule.npz")["rows"]
    for cos, warm, total, t, lr in rows:
        got = O.lr_at(int(t), 2e-5, int(warm), int(total), "cosine" if cos else "linear")
        assert got == lr
    assert O.lr_at(0, 2e-5, 3, 10, "cosine") == 0.0  # first step with warmup is a no-op


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "step_*.npz"))))
def test_step_block(path):
    z = np.load(path)
    wn, nmod, nsteps = int(z["world_size"]), int(z["n_modules"]), int(z["n_steps"])
    dt = str(z["dtype"])
    for j in range(nmod):
        W = z[f"r0.{j}.W0"]
        m = {k: [z[f"r{i}.s0.{j}.{k}_in"] for i in range(wn)] for k in ("m_A", "v_A", "m_B", "v_B")}
        A_l = [z[f"r{i}.{j}.A"] for i in range(wn)]
        B_l = [z[f"r{i}.{j}.B"] for i in range(wn)]
        for s in range(nsteps):
            t, lr = int(z[f"r0.s{s}.t"]), float(z[f"r0.s{s}.lr"])
            gA = [z[f"r{i}.s{s}.{j}.gA"] for i in range(wn)]
            gB = [z[f"r{i}.s{s}.{j}.gB"] for i in range(wn)]
            W_new, states, dW = O.step_module(gA, gB, m["m_A"], m["v_A"], m["m_B"], m["v_B"],
                                              A_l, B_l, W, t, lr, dt)
            for i in range(wn):
                for k, val in zip(("m_A", "v_A", "m_B", "v_B"), states[i]):
                    ref = z[f"r{i}.s{s}.{j}.{k}_out"]
                    assert O.rel_err(val, ref) < 1e-6, (path, s, j, i, k)
                    m[k][i] = ref
            if nmod == 1:
                ref_dW = z[f"r{wn - 1}.s{s}.0.dW"]
                tol = 1e-2 if dt == "bfloat16" else 1e-5
                assert O.rel_err(dW, ref_dW) < tol
                # delta of the last rank (the block's last loop-local values)
                _, _, dA_last = O.adam_factors(gA[-1], z[f"r{wn-1}.s{s}.0.m_A_in"], z[f"r{wn-1}.s{s}.0.v_A_in"], t, lr)
                assert O.rel_err(dA_last, z[f"r{wn-1}.s{s}.0.delta_A"]) < 1e-6
            for i in range(wn):
                W_ref = z[f"r{i}.s{s}.{j}.W"]
                # every rank holds the same merged weight
                assert np.array_equal(W_ref, z[f"r0.s{s}.{j}.W"])
            W_ref = z[f"r0.s{s}.{j}.W"]
            # merged-W parity: 1e-5 relative on the update itself (fp32), 2e-2 (bf16)
            upd = O.rel_err(W_new - W, W_ref - W)
            assert upd < (2e-2 if dt == "bfloat16" else 1e-4), (path, s, j, upd)
            assert O.rel_err(W_new, W_ref) < (2e-2 if dt == "bfloat16" else 1e-5)
            W = W_ref
