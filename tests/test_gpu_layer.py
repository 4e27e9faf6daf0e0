"""Layer / step parity on the GPU against golden vectors captured from the reference.

* probe_*.npz : CustomLinearLayer forward (== base linear) and the accumulated A.grad /
                B.grad after 3 micro-steps, through the real autograd path (K2).
* step_*.npz  : the literal hp:352-398 block's merged W_res and Adam moments after 3 steps.
                Wn = 1 runs the whole drop-in path (replace_with_custom_layer -> grads ->
                hd_pissa_step).  Wn > 1 on one GPU: every simulated rank's Adam (K3) runs on
                the device and the fused K = 2 r Wn gather-merge (K4) consumes all of them --
                exactly what each rank does after the all-gather.
"""
import glob
import os

import numpy as np
import pytest
import torch
import torch.nn as nn

from oracle import hdpissa_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _t(a, dtype=torch.float32):
    return torch.as_tensor(np.ascontiguousarray(a)).to(DEV).to(dtype)


def _np(t):
    return t.detach().float().cpu().numpy()


class FixtureSvdOps:
    """HIP ops, except svd_topk returns the reference's own factors (so Adam moments can be
    compared without sign alignment).  Factors are looked up by the weight's shape+sum."""

    def __init__(self, table):
        from hdpissa_amd.ops import default_ops
        self._hip = default_ops()
        self.table = table

    def __getattr__(self, k):
        return getattr(self._hip, k)

    def svd_topk(self, W, r, nranks):
        key = (tuple(W.shape), round(float(W.float().double().sum().item()), 6))
        return self.table[key]

    def svd_topk_batch(self, Ws, r, nranks):
        return [self.svd_topk(W, r, nranks) for W in Ws]


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "probe_*.npz"))))
def test_layer_probe_against_reference(path):
    from hdpissa_amd import CustomLinearLayer
    z = np.load(path)
    bf16 = "bf16" in path
    dt = torch.bfloat16 if bf16 else torch.float32
    out, inn = z["W"].shape
    r = int(z["r"])
    lin = nn.Linear(inn, out, bias="bias" in z.files).to(DEV)
    with torch.no_grad():
        lin.weight.copy_(_t(z["W"]))
        if "bias" in z.files:
            lin.bias.copy_(_t(z["bias"]))
    lin = lin.to(dt)
    for p in lin.parameters():
        p.requires_grad = False
    A_all = _t(z["A"])
    B_all = _t(z["B"])[None]
    layer = CustomLinearLayer(lin, "q_proj", 0, 1, r, float(z["alpha"]), 0.0, _factors=(A_all, B_all))
    assert layer.alpha == float(z["alpha_eff"])
    assert torch.equal(layer.W_res, lin.weight)
    for ms in range(3):
        x = _t(z[f"x{ms}"], dt)
        y = layer(x)
        ref_base = torch.nn.functional.linear(x, layer.W_res, layer.bias)
        assert torch.equal(y, ref_base)
        assert O.rel_err(_np(y), z[f"y{ms}"]) < (2e-2 if bf16 else 1e-5)
        y.backward(_t(z[f"G{ms}"], dt))
        if float(z["alpha_eff"]) == 0:
            assert not torch.any(layer.A.grad) and not torch.any(layer.B.grad)
            continue
        assert O.rel_err(_np(layer.A.grad), z[f"gA{ms}"]) < 1e-5, ms
        assert O.rel_err(_np(layer.B.grad), z[f"gB{ms}"]) < 1e-5, ms


def _step_files(wn):
    return sorted(glob.glob(os.path.join(GOLDEN, f"step_*_w{wn}.npz")))


class _Box(nn.Module):
    pass


def _build_model(z, j_specs, dt):
    """Container with modules named like the fixture's (layers.<i>.<proj>)."""
    root = _Box()
    root.layers = nn.ModuleList()
    table = {}
    for j, (name, out, inn, has_bias) in enumerate(j_specs):
        idx = int(name.split(".")[1])
        while len(root.layers) <= idx:
            root.layers.append(_Box())
        lin = nn.Linear(inn, out, bias=has_bias).to(DEV)
        with torch.no_grad():
            lin.weight.copy_(_t(z[f"r0.{j}.W0"]))
        lin = lin.to(dt)
        for p in lin.parameters():
            p.requires_grad = False
        setattr(root.layers[idx], name.split(".")[-1], lin)
        key = (tuple(lin.weight.shape), round(float(lin.weight.float().double().sum().item()), 6))
        table[key] = (_t(z[f"r0.{j}.A"]), _t(z[f"r0.{j}.B"])[None], None)
    return root, table


STEP_SPECS = {
    "f32_tall": [("layers.0.q_proj", 64, 48, True)],
    "f32_wide": [("layers.0.down_proj", 40, 72, False)],
    "bf16_tall": [("layers.0.q_proj", 64, 48, True)],
    "f32_two": [("layers.0.q_proj", 48, 48, False), ("layers.1.up_proj", 64, 32, False)],
}


@pytest.mark.parametrize("exchange", ["gather", "allreduce"])
@pytest.mark.parametrize("path", _step_files(1))
def test_step_wn1_drop_in(path, exchange):
    from hdpissa_amd import HDPissaStep, replace_with_custom_layer
    z = np.load(path)
    case = os.path.basename(path)[5:-7]
    specs = STEP_SPECS[case]
    dt = torch.bfloat16 if str(z["dtype"]) == "bfloat16" else torch.float32
    model, table = _build_model(z, specs, dt)
    layers = replace_with_custom_layer(model, [s[0].split(".")[-1] for s in specs], 0, 1, int(z["r"]),
                                       float(z["alpha"]), ops=FixtureSvdOps(table))
    stepper = HDPissaStep(model, 1, 0, exchange=exchange)
    for s in range(int(z["n_steps"])):
        for j, L in enumerate(layers):
            L.A.grad = _t(z[f"r0.s{s}.{j}.gA"])
            L.B.grad = _t(z[f"r0.s{s}.{j}.gB"])
        stepper.step(float(z[f"r0.s{s}.lr"]), int(z[f"r0.s{s}.t"]))
        torch.cuda.synchronize()
        for j, L in enumerate(layers):
            assert L.A.grad is None and L.B.grad is None
            W_prev = z[f"r0.{j}.W0"] if s == 0 else z[f"r0.s{s - 1}.{j}.W"]
            W_ref = z[f"r0.s{s}.{j}.W"]
            got = _np(L.W_res)
            if dt == torch.float32:
                assert O.rel_err(got, W_ref) < 1e-6
                assert O.rel_err(got - W_prev, W_ref - W_prev) < 1e-4
            else:
                # W alone would pass even with the step skipped (one update is ~1.3 % of ||W||):
                # check the update, and the reference's bf16 rounding (at Wn = 1 both exchanges
                # round dW once, then W + dW once, as hp:389-394 does) element for element
                assert O.rel_err(got, W_ref) < 2e-2
                assert O.rel_err(got - W_prev, W_ref - W_prev) < 2e-2
                assert np.mean(got != W_ref) < 0.02
            for k in ("m_A", "v_A", "m_B", "v_B"):
                assert O.rel_err(_np(getattr(L, k)), z[f"r0.s{s}.{j}.{k}_out"]) < 1e-6
            # continue from the reference's W (keeps the comparison per-step)
            with torch.no_grad():
                L.W_res.copy_(_t(W_ref, dt))


@pytest.mark.parametrize("path", _step_files(2) + _step_files(4))
def test_step_multirank_simulated(path):
    """Every simulated rank's Adam on the GPU, then the K = 2 r Wn fused gather-merge."""
    from hdpissa_amd.ops import default_ops
    from hdpissa_amd._lib import HDP_DW_MERGE
    ops = default_ops()
    z = np.load(path)
    wn, nmod = int(z["world_size"]), int(z["n_modules"])
    dt = torch.bfloat16 if str(z["dtype"]) == "bfloat16" else torch.float32
    for j in range(nmod):
        A = [z[f"r{i}.{j}.A"] for i in range(wn)]
        B = [z[f"r{i}.{j}.B"] for i in range(wn)]
        r, inn = A[0].shape
        out = B[0].shape[0]
        F = r * inn + out * r
        fac = torch.zeros(wn, F, device=DEV)
        for i in range(wn):
            fac[i, :r * inn] = _t(A[i]).reshape(-1)
            fac[i, r * inn:] = _t(B[i]).reshape(-1)
        m = torch.zeros(wn, F, device=DEV)
        v = torch.zeros(wn, F, device=DEV)
        W = _t(z[f"r0.{j}.W0"], dt)
        for s in range(int(z["n_steps"])):
            t, lr = int(z[f"r0.s{s}.t"]), float(z[f"r0.s{s}.lr"])
            delta = torch.zeros(wn, F, device=DEV)
            for i in range(wn):
                g = torch.cat([_t(z[f"r{i}.s{s}.{j}.gA"]).reshape(-1), _t(z[f"r{i}.s{s}.{j}.gB"]).reshape(-1)])
                ops.adam(g, m[i], v[i], delta[i], t, lr, 0.9, 0.999, 1e-8, zero_grad=True)
            flat_d, flat_f = delta.view(-1), fac.view(-1)
            ops.delta_gemm(out, inn, r, wn, flat_d, flat_d[r * inn:], F, flat_f, flat_f[r * inn:], F, W,
                           HDP_DW_MERGE, dt == torch.bfloat16)
            torch.cuda.synchronize()
            for i in range(wn):
                assert O.rel_err(_np(m[i, :r * inn]).reshape(r, inn), z[f"r{i}.s{s}.{j}.m_A_out"]) < 1e-6
                assert O.rel_err(_np(v[i, r * inn:]).reshape(out, r), z[f"r{i}.s{s}.{j}.v_B_out"]) < 1e-6
            W_ref = z[f"r0.s{s}.{j}.W"]
            W_prev = z[f"r0.{j}.W0"] if s == 0 else z[f"r0.s{s - 1}.{j}.W"]
            got = _np(W)
            if dt == torch.float32:
                assert O.rel_err(got, W_ref) < 1e-6
                assert O.rel_err(got - W_prev, W_ref - W_prev) < 1e-4
            else:
                assert O.rel_err(got, W_ref) < 2e-2
                assert np.mean(got != W_ref) < 0.02
            W.copy_(_t(W_ref, dt))


def test_native_probe_queue_groups_and_accumulates():
    """The native hdp_probe_queue behind ProbeQueue: several layers, repeated modules inside one
    pass (forces a flush), a byte budget small enough to split groups, two dtypes' worth of
    queues not needed here -- accumulated A.grad / B.grad equal the oracle's sums."""
    from hdpissa_amd import flush_probes, replace_with_custom_layer
    g = np.random.default_rng(7)
    shapes = [(96, 64), (64, 96), (128, 64), (64, 64), (160, 96)]
    root = _Box()
    for i, (out, inn) in enumerate(shapes):
        lin = nn.Linear(inn, out, bias=False).to(DEV)
        for p in lin.parameters():
            p.requires_grad = False
        setattr(root, f"p{i}_proj", lin)
    layers = replace_with_custom_layer(root, ["_proj"], 0, 1, 8, 8.0)
    q = layers[0]._arena.probe_queue
    q.budget = 200_000  # a few modules per group
    ref = [(np.zeros((8, L.in_features)), np.zeros((L.out_features, 8))) for L in layers]
    order = [0, 1, 2, 0, 3, 4, 4, 1, 2, 3, 0]  # repeats inside the sequence -> flushes
    for rep in range(3):
        for i in order:
            L = layers[i]
            T = int(g.integers(1, 70))
            X = g.standard_normal((T, L.in_features)).astype(np.float32)
            G = g.standard_normal((T, L.out_features)).astype(np.float32)
            L._probe_backward(_t(X), _t(G))
            gA, gB = O.probe_grads(X, G, _np(L.A), _np(L.B), O.alpha_eff(8.0, 8))
            ref[i] = (ref[i][0] + gA.astype(np.float64), ref[i][1] + gB.astype(np.float64))
    flush_probes(root)
    torch.cuda.synchronize()
    assert q._nq, "the native queue was not used"
    for L, (gA, gB) in zip(layers, ref):
        assert O.rel_err(_np(L.A.grad), gA) < 1e-5
        assert O.rel_err(_np(L.B.grad), gB) < 1e-5
    assert sum(h.flushes() for h in q._nq.values()) >= 6


def test_probe_queue_mixed_dtypes_keep_push_order():
    """f32 and bf16 activations pushed into one arena: one native queue per X dtype, but the
    groups launch in push order (a later overwrite never overtakes an earlier accumulate) and
    every pending operand stays alive until its group is launched."""
    from hdpissa_amd import flush_probes, replace_with_custom_layer
    g = np.random.default_rng(17)
    shapes = [(96, 64), (64, 128), (128, 64)]
    root = _Box()
    for i, (out, inn) in enumerate(shapes):
        lin = nn.Linear(inn, out, bias=False).to(DEV)
        for p in lin.parameters():
            p.requires_grad = False
        setattr(root, f"p{i}_proj", lin)
    layers = replace_with_custom_layer(root, ["_proj"], 0, 1, 8, 8.0)
    ref = [None] * len(layers)
    seq = [(0, "f32"), (1, "f32"), (0, "bf16"), (2, "bf16"), (1, "f32"), (2, "f32"), (0, "bf16")]
    for i, kind in seq:
        L = layers[i]
        T = int(g.integers(5, 40))
        X = g.standard_normal((T, L.in_features)).astype(np.float32)
        G = g.standard_normal((T, L.out_features)).astype(np.float32)
        if kind == "bf16":
            X, G = O.round_bf16(X), O.round_bf16(G)
        dt = torch.bfloat16 if kind == "bf16" else torch.float32
        if ref[i] is None:  # the first backward of a layer overwrites (A.grad is None)
            L.A.grad = None
            L.B.grad = None
        L._probe_backward(_t(X, dt), _t(G, dt))
        gA, gB = O.probe_grads(X, G, _np(L.A), _np(L.B), O.alpha_eff(8.0, 8))
        ref[i] = (gA, gB) if ref[i] is None else (ref[i][0] + gA, ref[i][1] + gB)
        torch.cuda.empty_cache()  # would hand freed memory to new tensors if a pending X/G were dropped
        _ = torch.randn(1 << 18, device=DEV)
    flush_probes(root)
    torch.cuda.synchronize()
    for L, (gA, gB) in zip(layers, ref):
        assert O.rel_err(_np(L.A.grad), gA) < 1e-5
        assert O.rel_err(_np(L.B.grad), gB) < 1e-5


def test_native_push_fallbacks():
    """The one-call native push (_C.LayerSlot) hands every case it does not own back to the Python
    path: B edited in place (B^T re-cached), A replaced by a new Parameter, one grad cleared by the
    user, and a second activation dtype -- accumulated grads still equal the oracle's."""
    from hdpissa_amd import flush_probes, replace_with_custom_layer
    g = np.random.default_rng(23)
    root = _Box()
    lin = nn.Linear(64, 96, bias=False).to(DEV)
    lin.weight.requires_grad = False
    root.q_proj = lin
    (L,) = replace_with_custom_layer(root, ["q_proj"], 0, 1, 8, 8.0)
    s = O.alpha_eff(8.0, 8)

    def push(dt=torch.float32):
        X = g.standard_normal((9, 64)).astype(np.float32)
        G = g.standard_normal((9, 96)).astype(np.float32)
        if dt == torch.bfloat16:
            X, G = O.round_bf16(X), O.round_bf16(G)
        L._probe_backward(_t(X, dt), _t(G, dt))
        return O.probe_grads(X, G, _np(L.A), _np(L.B), s)

    def check(eA, eB):
        flush_probes(root)
        torch.cuda.synchronize()
        assert O.rel_err(_np(L.A.grad), eA) < 1e-5
        assert O.rel_err(_np(L.B.grad), eB) < 1e-5

    eA, eB = push()
    a, b = push()  # the fast path (LayerSlot registered by the first push)
    assert L._fslot is not None
    check(eA + a, eB + b)
    eA, eB = eA + a, eB + b
    with torch.no_grad():
        L.B.mul_(1.5)  # in place: version bump -> B^T re-cached
    a, b = push()
    check(eA + a, eB + b)
    eA, eB = eA + a, eB + b
    L.B.grad = None  # user clears one grad: B restarts at zero, A accumulates
    a, b = push()
    check(eA + a, b)
    eA, eB = eA + a, b
    L.A = nn.Parameter(L.A.detach().clone())  # replaced (no longer the arena view)
    L.A.grad = L._gA
    a, b = push()
    check(eA + a, eB + b)
    eA, eB = eA + a, eB + b
    a, b = push(torch.bfloat16)  # second dtype: pushes go through the Python path in order
    a2, b2 = push()
    check(eA + a + a2, eB + b + b2)


def test_probe_unaligned_activation_view():
    """A contiguous activation view at a 4-byte storage offset: re-based, not rejected."""
    from hdpissa_amd import flush_probes, replace_with_custom_layer
    root = _Box()
    lin = nn.Linear(64, 96, bias=False).to(DEV)
    lin.weight.requires_grad = False
    root.q_proj = lin
    (L,) = replace_with_custom_layer(root, ["q_proj"], 0, 1, 8, 8.0)
    T = 12
    bx = torch.randn(T * 64 + 1, device=DEV)
    bg = torch.randn(T * 96 + 1, device=DEV)
    X, G = bx[1:].view(T, 64), bg[1:].view(T, 96)
    assert X.data_ptr() % 16 and G.data_ptr() % 16
    L._probe_backward(X, G)
    flush_probes(root)
    torch.cuda.synchronize()
    gA, gB = O.probe_grads(_np(X), _np(G), _np(L.A), _np(L.B), O.alpha_eff(8.0, 8))
    assert O.rel_err(_np(L.A.grad), gA) < 1e-5
    assert O.rel_err(_np(L.B.grad), gB) < 1e-5


@pytest.mark.parametrize("dt", ["float32", "bfloat16"])
@pytest.mark.parametrize("wn", [1, 4])
def test_pissa_residual_mode_gpu(dt, wn):
    """Opt-in PiSSA-residual mode on the device: W_res = W - sum_i B_i A_i formed by the grouped
    delta GEMM (K4, MERGE, dA := A), vs the float64 oracle; merged weight == W; the forward equals
    the default mode's."""
    from hdpissa_amd import replace_with_custom_layer
    tdt = torch.bfloat16 if dt == "bfloat16" else torch.float32
    outs = {}
    for residual in (False, True):
        torch.manual_seed(5)
        root = _Box()
        for i, (out, inn) in enumerate([(256, 192), (160, 320), (512, 512)]):
            lin = nn.Linear(inn, out, bias=(i == 0)).to(DEV).to(tdt)
            for p in lin.parameters():
                p.requires_grad = False
            setattr(root, f"p{i}_proj", lin)
        W0 = {n: m.weight.detach().float().cpu().numpy() for n, m in root.named_modules() if isinstance(m, nn.Linear)}
        layers = replace_with_custom_layer(root, ["_proj"], 0, wn, 16, 16.0, residual=residual)
        torch.cuda.synchronize()
        x = torch.randn(4, 7, 192, device=DEV).to(tdt)
        outs[residual] = root.p0_proj(x).detach().float().cpu().numpy()
        if residual:
            for L in layers:
                a = L._arena
                i = a.layers.index(L)
                A = [_np(a.views(a.fac_all[d], i)[0]) for d in range(wn)]
                B = [_np(a.views(a.fac_all[d], i)[1]) for d in range(wn)]
                ref = O.pissa_residual(W0[L.name], A, B)
                got = _np(L.W_res)
                if dt == "float32":
                    assert O.rel_err(got, ref) < 1e-6
                else:
                    # bf16 W_res: the merge's rounding (W + bf16(-sum_i B_i A_i), like hp:394's cast)
                    ref16 = O.merge(W0[L.name], (ref - W0[L.name]).astype(np.float32), "bfloat16")
                    assert O.rel_err(got, ref) < 2e-2 and np.mean(got != ref16) < 0.02
                assert O.rel_err(_np(L.merge_weights()), W0[L.name]) < (1e-6 if dt == "float32" else 2e-2)
    assert O.rel_err(outs[True], outs[False]) < (1e-5 if dt == "float32" else 2e-2)
