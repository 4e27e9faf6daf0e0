"""K2 parity at the bench's own decoder-layer layouts (hp:139 + autograd).

The headline bench feeds the probe the way a decoder's autograd does: q/k/v read ONE saved hidden state,
gate/up ONE, o and down their own (bench.py: one X per projection group, row views X[:T] of a resident
buffer).  So the sweep runs its shared-X FUSE instances -- phase A's X6 form for float32 activations,
the FUSE OUTER phase C -- over sets whose X is 4096 / 5120 wide with outs up to 14336, which the
reduced-width shared-X test (test_gpu_kernels.py::test_probe_shared_x_sets, 1024 / 2752) never reaches.

For each BASELINE layer layout (LLaMA-2-7B f32 r16, Mistral-7B bf16 r64 with k/v 1024 beside q 4096,
LLaMA-2-13B bf16 r128 = two r-slices of 64, Qwen2.5-0.5B f32 r16 with kv 128), at T = 691 (the bench's
mean padded micro-batch), 1024 (the longest) and 17 (ragged, one partial 16-row step):

* through the group API (hdp_probe_grads_group), members accumulating or overwriting, vs the float64
  oracle (O.probe_grads) at 1e-5 relative -- the bar of every K2 test (bf16 activations are exact in
  bf16 and the kernel's products reach f32 resolution);
* through the layer path the bench drives (CustomLinearLayer._probe_backward -> native queue, then
  _C.LayerSlot.push per module backward): three micro-batches accumulated into A.grad / B.grad, then a
  fourth after the grads were cleared (overwrite: the arena's stale gradient must not leak in).
"""
import numpy as np
import pytest
import torch

from oracle import hdpissa_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"

# layout -> (model dtype, r, hidden, intermediate, kv width)
LAYOUTS = {
    "llama2-7b": ("float32", 16, 4096, 11008, 4096),
    "mistral-7b": ("bfloat16", 64, 4096, 14336, 1024),
    "llama2-13b": ("bfloat16", 128, 5120, 13824, 5120),
    "qwen2.5-0.5b": ("float32", 16, 896, 4864, 128),
}
TS = (691, 1024, 17)
TOL = 1e-5


def _mods(H, I, KV):
    # (name, X group, out, in) in the bench's module order
    return [("q_proj", "attn", H, H), ("k_proj", "attn", KV, H), ("v_proj", "attn", KV, H), ("o_proj", "o", H, H),
            ("gate_proj", "mlp", I, H), ("up_proj", "mlp", I, H), ("down_proj", "down", H, I)]


def _np(t):
    return t.detach().double().cpu().numpy()


def _inputs(layout, seed):
    """Resident X per projection group and G per module (Tmax rows), as the bench lays them out."""
    dt, r, H, I, KV = LAYOUTS[layout]
    tdt = getattr(torch, dt)
    g = torch.Generator(device=DEV).manual_seed(seed)
    Tm = max(TS)
    xs, gs = {}, {}
    for name, grp, out, inn in _mods(H, I, KV):
        if grp not in xs:
            xs[grp] = torch.empty(Tm, inn, device=DEV).normal_(generator=g).to(tdt)
        gs[name] = torch.empty(Tm, out, device=DEV).normal_(0, 1e-3, generator=g).to(tdt)
    return xs, gs


@pytest.fixture(scope="module")
def ops():
    from hdpissa_amd.ops import default_ops
    return default_ops()


@pytest.mark.parametrize("layout", list(LAYOUTS))
def test_probe_group_layer_layout(ops, layout):
    """One decoder layer's seven modules in ONE group call, X shared by pointer like autograd saves it."""
    from hdpissa_amd._lib import lib
    dt, r, H, I, KV = LAYOUTS[layout]
    xs, gs = _inputs(layout, 11)
    g = torch.Generator(device=DEV).manual_seed(12)
    mods = _mods(H, I, KV)
    fac = {}
    for name, _, out, inn in mods:
        A = torch.randn(r, inn, device=DEV, generator=g) * 0.05
        B = torch.randn(out, r, device=DEV, generator=g) * 0.05
        fac[name] = (A, B, B.t().contiguous())
    assert lib().hdp_probe_errors(1) == 0
    for T in TS:
        items, refs = [], []
        for j, (name, grp, out, inn) in enumerate(mods):
            A, B, Bt = fac[name]
            acc = (j + T) % 2 == 0  # members mix accumulate / overwrite
            gA0 = torch.randn(r, inn, device=DEV, generator=g) * 1e-16
            gB0 = torch.randn(out, r, device=DEV, generator=g) * 1e-16
            X, G = xs[grp][:T], gs[name][:T]
            items.append((X, G, A, Bt, gA0, gB0, 3e-16, acc))
            refs.append((name, X, G, A, B, _np(gA0) if acc else 0.0, _np(gB0) if acc else 0.0))
        ops.probe_grads_group(items)
        torch.cuda.synchronize()
        assert lib().hdp_probe_errors(1) == 0, (layout, T)
        for it, (name, X, G, A, B, a0, b0) in zip(items, refs):
            eA, eB = O.probe_grads(_np(X), _np(G), _np(A), _np(B), 1.0)
            errA = O.rel_err(_np(it[4]), a0 + 3.0 * eA)
            errB = O.rel_err(_np(it[5]), b0 + 3.0 * eB)
            assert errA < TOL and errB < TOL, (layout, T, name, errA, errB)


@pytest.mark.parametrize("layout", list(LAYOUTS))
def test_probe_layer_path_layer_layout(layout):
    """The path bench.py times: replace_with_custom_layer on one decoder layer, module backward per
    micro-batch through _probe_backward (the native LayerSlot push after the first), flush."""
    import bench
    from hdpissa_amd import flush_probes, replace_with_custom_layer
    from hdpissa_amd._lib import lib
    from hdpissa_amd.ops import default_ops
    dt, r, H, I, KV = LAYOUTS[layout]
    wl = dict(bench.WORKLOADS[layout], layers=1)
    model, targets = bench.build_model(wl, torch.device(DEV))
    layers = replace_with_custom_layer(model, targets, 0, 1, r, float(r), ops=bench._RandomFactorOps(default_ops()))
    xs, gs = _inputs(layout, 21)
    grp = {name: g for name, g, _, _ in _mods(H, I, KV)}
    assert lib().hdp_probe_errors(1) == 0

    def micro(T):
        for L in layers:
            name = L.name.rsplit(".", 1)[1]
            L._probe_backward(xs[grp[name]][:T], gs[name][:T])

    def expect(Ts):
        out = {}
        for L in layers:
            name = L.name.rsplit(".", 1)[1]
            A, B = _np(L.A), _np(L.B)
            eA = eB = 0.0
            for T in Ts:
                a, b = O.probe_grads(_np(xs[grp[name]][:T]), _np(gs[name][:T]), A, B, L.alpha)
                eA, eB = eA + a, eB + b
            out[L.name] = (eA, eB)
        return out

    for T in TS:  # accumulate over three micro-batches (the first call registers the native slot)
        micro(T)
    flush_probes(model)
    torch.cuda.synchronize()
    assert lib().hdp_probe_errors(1) == 0
    ref = expect(TS)
    for L in layers:
        eA, eB = ref[L.name]
        errA, errB = O.rel_err(_np(L.A.grad), eA), O.rel_err(_np(L.B.grad), eB)
        assert errA < TOL and errB < TOL, (layout, "accumulate", L.name, errA, errB)
    for L in layers:  # what the step leaves (hp:397-398): the next backward overwrites
        L.A.grad = None
        L.B.grad = None
    micro(691)
    flush_probes(model)
    torch.cuda.synchronize()
    ref = expect((691,))
    for L in layers:
        eA, eB = ref[L.name]
        errA, errB = O.rel_err(_np(L.A.grad), eA), O.rel_err(_np(L.B.grad), eB)
        assert errA < TOL and errB < TOL, (layout, "overwrite", L.name, errA, errB)
