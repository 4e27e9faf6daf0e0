"""CPU stand-in for the HIP op set -- TEST INFRASTRUCTURE ONLY.

Lets the CPU suite drive the product host logic (arena layout, bucket plans, both exchange
strategies, multi-rank orchestration under gloo) without a GPU.  It is injected explicitly
(``ops=CpuOps()``); the product never selects it, and ``hdpissa_amd.ops.HipOps`` raises on
CPU tensors.  Semantics follow the oracle (and the kernels' documented contract).
"""
import numpy as np
import torch

from oracle import hdpissa_oracle as O


def _seg(t, i, stride, n, shape):
    return t.reshape(-1)[i * stride:i * stride + n].view(*shape)


class CpuOps:
    name = "cpu-test"

    def __init__(self, factors=None):
        self.factors = factors  # optional {key: (A_all, B_all)} keyed like FixtureSvdOps

    def svd_topk(self, W, r, nranks):
        if self.factors is not None:
            key = (tuple(W.shape), round(float(W.float().double().sum().item()), 6))
            A_all, B_all = self.factors[key]
            return A_all.clone(), B_all.clone(), None
        k = r * nranks
        if k > min(W.shape):
            raise ValueError("ranks_per_gpu * world_size exceeds min(out, in)")
        U, S, V = O.svd_full(W.float().numpy())
        sq = np.sqrt(S[:k])
        A_all = torch.from_numpy((sq[:, None] * V[:, :k].T).astype(np.float32))
        B = (U[:, :k] * sq[None, :]).astype(np.float32)
        B_all = torch.from_numpy(np.ascontiguousarray(B.reshape(W.shape[0], nranks, r).transpose(1, 0, 2)))
        return A_all, B_all, torch.from_numpy(S[:k])

    def probe_grads(self, X, G, A, B, gA, gB, scale, accumulate, Bt=None):
        if Bt is not None:
            assert torch.equal(Bt, B.t())
        X64, G64 = X.double(), G.double()
        H = X64 @ A.double().T
        J = G64 @ B.double()
        dA = (J.T @ X64).float() * np.float32(scale)
        dB = (G64.T @ H).float() * np.float32(scale)
        if accumulate:
            gA.add_(dA)
            gB.add_(dB)
        else:
            gA.copy_(dA)
            gB.copy_(dB)

    def probe_group_max(self):
        return 16

    def probe_grads_group(self, items):
        ids = set()
        for X, G, A, Bt, gA, gB, scale, acc in items:
            assert id(gA) not in ids
            ids.add(id(gA))
            self.probe_grads(X, G, A, Bt.t(), gA, gB, scale, acc)

    def adam(self, grad, m, v, delta, t, lr, beta1, beta2, eps, zero_grad, grad_scale=1e16):
        mn, vn, d = O.adam_factors(grad.numpy(), m.numpy(), v.numpy(), t, lr, beta1, beta2, eps)
        m.copy_(torch.from_numpy(mn))
        v.copy_(torch.from_numpy(vn))
        delta.copy_(torch.from_numpy(d))
        if zero_grad:
            grad.zero_()

    def delta_gemm(self, out, inn, r, nseg, dA, dB, delta_stride, A, B, factor_stride, dst, mode, round_bf16):
        run = torch.zeros(out, inn)
        for i in range(nseg):
            a = _seg(A, i, factor_stride, r * inn, (r, inn))
            b = _seg(B, i, factor_stride, out * r, (out, r))
            da = _seg(dA, i, delta_stride, r * inn, (r, inn))
            db = _seg(dB, i, delta_stride, out * r, (out, r))
            run = run - (db @ (a - da) + b @ da)
            if round_bf16:
                run = run.bfloat16().float()
        d = dst.reshape(-1)[:out * inn].view(out, inn)
        if mode == 0:
            d.copy_(run)
        elif d.dtype == torch.bfloat16:
            d.copy_((d.float() + run.bfloat16().float()).bfloat16())
        else:
            d.add_(run)

    def delta_plan(self, items, mode, round_bf16):
        ops = self

        class _Plan:
            n = len(items)

            def valid(self, dsts=None):
                return True

            def run(self):
                for it in items:
                    ops.delta_gemm(*it, mode, round_bf16)

        return _Plan()

    def fold_bf16(self, parts, out):
        run = torch.zeros(parts.shape[1])
        for i in range(parts.shape[0]):
            run = (run + parts[i]).bfloat16().float()  # float32 sum, then the bf16 cast (hp:392)
        out.copy_(run.bfloat16())

    def merge(self, W, dW):
        if W.dtype == torch.bfloat16:
            W.copy_((W.float() + dW.view_as(W).bfloat16().float()).bfloat16())
        else:
            W.add_(dW.view_as(W))
