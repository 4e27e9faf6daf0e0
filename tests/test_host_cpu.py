"""Host-side logic on CPU: the drop-in API surface, arena layout, bucket planning, both
exchange strategies and error behaviour.  Arithmetic comes from the test-only CpuOps (the
product's HIP ops refuse CPU tensors -- checked here too)."""
import glob
import os

import numpy as np
import pytest
import torch
import torch.nn as nn

from cpu_ops import CpuOps
from helpers import build_fixture_model, rel_err
from oracle import hdpissa_oracle as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_hip_ops_refuse_cpu_tensors():
    from hdpissa_amd._lib import LIB_PATH
    if not os.path.exists(LIB_PATH):
        pytest.skip("library not built")
    from hdpissa_amd.ops import HipOps
    ops = HipOps()
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        ops.merge(torch.zeros(4), torch.zeros(4))
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        ops.svd_topk(torch.zeros(8, 8), 2, 1)


def test_missing_library_fails_loudly(monkeypatch):
    import hdpissa_amd._lib as L
    monkeypatch.setattr(L, "_lib", None)
    monkeypatch.setattr(L, "LIB_PATH", "/nonexistent/libhdpissa.so")
    with pytest.raises(L.HdpLibraryError):
        L.lib()


def _tiny_model():
    m = nn.Module()
    m.model = nn.Module()
    m.model.layers = nn.ModuleList([nn.Module() for _ in range(2)])
    for i, blk in enumerate(m.model.layers):
        blk.self_attn = nn.Module()
        blk.self_attn.q_proj = nn.Linear(32, 32, bias=True)
        blk.self_attn.o_proj = nn.Linear(32, 32, bias=False)
        blk.mlp = nn.Module()
        blk.mlp.down_proj = nn.Linear(48, 32, bias=False)
        blk.mlp.act = nn.GELU()
    for p in m.parameters():
        p.requires_grad = False
    return m


def test_replace_matches_reference_targeting():
    from hdpissa_amd import CustomLinearLayer, custom_layers, replace_with_custom_layer
    m = _tiny_model()
    layers = replace_with_custom_layer(m, ["q_proj", "down_proj"], 0, 1, 4, 16.0, ops=CpuOps())
    names = [n for n, _ in custom_layers(m)]
    assert names == ["model.layers.0.self_attn.q_proj", "model.layers.0.mlp.down_proj",
                     "model.layers.1.self_attn.q_proj", "model.layers.1.mlp.down_proj"]
    assert isinstance(m.model.layers[0].self_attn.o_proj, nn.Linear)
    L = layers[0]
    assert repr(L) == "CustomLinearLayer(name=model.layers.0.self_attn.q_proj, in_features=32, out_features=32)"
    assert L.alpha == 4.0 and L.A.shape == (4, 32) and L.B.shape == (32, 4)
    assert L.A.dtype == torch.float32 and L.A.requires_grad
    assert L.dropout_rate == 0.0 and isinstance(L.dropout, nn.Dropout)
    assert L.bias is not None and layers[1].bias is None
    # all layers share one arena; factors are aligned views
    arena = L._arena
    assert all(x._arena is arena for x in layers)
    for x in layers:
        base = arena.fac.data_ptr()
        assert (x.A.data_ptr() - base) % 256 == 0 and (x.B.data_ptr() - base) % 256 == 0
        assert x.m_A.shape == x.A.shape and x.v_B.shape == x.B.shape
    merged = L.merge_weights()
    assert torch.equal(merged, L.W_res) and merged.data_ptr() != L.W_res.data_ptr()


def test_reference_error_behaviour():
    from hdpissa_amd import CustomLinearLayer, replace_with_custom_layer
    lin = nn.Linear(16, 8)
    with pytest.raises(TypeError):  # hp:103 fails on ranks_per_gpu=None
        CustomLinearLayer(lin, "q", 0, 1, None, 16.0, ops=CpuOps())
    with pytest.raises(ValueError):  # more triplets than singular values
        replace_with_custom_layer(nn.ModuleDict({"q_proj": lin}), ["q_proj"], 0, 4, 4, 16.0, ops=CpuOps())
    with pytest.raises(NotImplementedError):
        CustomLinearLayer(lin, "q", 0, 1, 2, 16.0, dropout=0.1, ops=CpuOps())


def test_alpha_floor_division():
    from hdpissa_amd import CustomLinearLayer
    lin = nn.Linear(16, 8)
    assert CustomLinearLayer(lin, "q", 0, 1, 4, 3.0, ops=CpuOps()).alpha == 0.0
    assert CustomLinearLayer(lin, "q", 0, 1, 4, 7.0, ops=CpuOps()).alpha == 1.0
    assert CustomLinearLayer(lin, "q", 0, 1, 64 // 16, 16.0, ops=CpuOps()).alpha == 4.0


def test_svd_slice_cpu_ops_match_oracle():
    """CpuOps' factor layout (A_all rows per rank, B_all slabs) is the C-ABI's."""
    g = np.random.default_rng(0)
    W = g.standard_normal((24, 20)).astype(np.float32)
    A_all, B_all, _ = CpuOps().svd_topk(torch.from_numpy(W), 3, 2)
    for d in range(2):
        A, B, _, _ = O.svd_slice(W, d, 2, 3)
        assert rel_err(A_all[3 * d:3 * d + 3].numpy(), A) < 1e-6
        assert rel_err(B_all[d].numpy(), B) < 1e-6


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "probe_*.npz"))))
def test_probe_autograd_path(path):
    from hdpissa_amd import CustomLinearLayer
    z = np.load(path)
    bf16 = "bf16" in path
    dt = torch.bfloat16 if bf16 else torch.float32
    out, inn = z["W"].shape
    lin = nn.Linear(inn, out, bias="bias" in z.files)
    with torch.no_grad():
        lin.weight.copy_(torch.from_numpy(z["W"]))
        if "bias" in z.files:
            lin.bias.copy_(torch.from_numpy(z["bias"]))
    lin = lin.to(dt).requires_grad_(False)
    L = CustomLinearLayer(lin, "q_proj", 0, 1, int(z["r"]), float(z["alpha"]), ops=CpuOps(),
                          _factors=(torch.from_numpy(z["A"]), torch.from_numpy(z["B"])[None]))
    for ms in range(3):
        x = torch.from_numpy(z[f"x{ms}"]).to(dt)
        y = L(x)
        assert torch.equal(y, torch.nn.functional.linear(x, L.W_res, L.bias))
        y.backward(torch.from_numpy(z[f"G{ms}"]).to(dt))
        assert L.A.grad.data_ptr() == L._gA.data_ptr()  # grads land in the arena
        if float(z["alpha_eff"]) == 0:
            assert not torch.any(L.A.grad)
            continue
        assert rel_err(L.A.grad.numpy(), z[f"gA{ms}"]) < 1e-5
        assert rel_err(L.B.grad.numpy(), z[f"gB{ms}"]) < 1e-5


def test_bucket_plan():
    from hdpissa_amd.step import _buckets
    assert _buckets([5, 5, 5, 5], 10) == [(0, 2), (2, 4)]
    assert _buckets([20, 1, 1], 10) == [(0, 1), (1, 3)]
    assert _buckets([3], 1) == [(0, 1)]
    assert _buckets([], 4) == []


@pytest.mark.parametrize("exchange", ["gather", "allreduce"])
@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "step_*_w1.npz"))))
def test_step_wn1_host(path, exchange):
    from hdpissa_amd import HDPissaStep, replace_with_custom_layer
    from hdpissa_amd.comm import LocalComm
    z = np.load(path)
    case = os.path.basename(path)[5:-7]
    model, table, targets, dt = build_fixture_model(z, case)
    ops = CpuOps(table)
    layers = replace_with_custom_layer(model, targets, 0, 1, int(z["r"]), float(z["alpha"]), ops=ops)
    st = HDPissaStep(model, 1, 0, comm=LocalComm(), ops=ops, exchange=exchange, bucket_bytes=4096)
    for s in range(int(z["n_steps"])):
        for j, L in enumerate(layers):
            L.A.grad = torch.from_numpy(z[f"r0.s{s}.{j}.gA"])
            L.B.grad = torch.from_numpy(z[f"r0.s{s}.{j}.gB"])
        st.step(float(z[f"r0.s{s}.lr"]), int(z[f"r0.s{s}.t"]))
        for j, L in enumerate(layers):
            assert L.A.grad is None
            W_ref = z[f"r0.s{s}.{j}.W"]
            got = L.W_res.float().numpy()
            assert rel_err(got, W_ref) < (2e-2 if dt == torch.bfloat16 else 1e-6)
            for k in ("m_A", "v_A", "m_B", "v_B"):
                assert rel_err(getattr(L, k).numpy(), z[f"r0.s{s}.{j}.{k}_out"]) < 1e-6
            with torch.no_grad():
                L.W_res.copy_(torch.from_numpy(W_ref).to(dt))


def test_lr_schedule_product_matches_golden():
    from hdpissa_amd import lr_at
    rows = np.load(os.path.join(GOLDEN, "lr_schedule.npz"))["rows"]
    for cos, warm, total, t, lr in rows:
        assert lr_at(int(t), 2e-5, int(warm), int(total), "cosine" if cos else "linear") == lr


def test_save_custom_model_roundtrip(tmp_path):
    transformers = pytest.importorskip("transformers")
    from hdpissa_amd import replace_with_custom_layer, save_custom_model
    cfg = transformers.Qwen2Config(hidden_size=32, intermediate_size=64, num_hidden_layers=1, num_attention_heads=4,
                                   num_key_value_heads=2, vocab_size=64, max_position_embeddings=32)
    model = transformers.Qwen2ForCausalLM(cfg)
    for p in model.parameters():
        p.requires_grad = False
    layers = replace_with_custom_layer(model, ["q_proj", "down_proj"], 0, 1, 2, 4.0, ops=CpuOps())
    with torch.no_grad():
        layers[0].W_res.add_(1.0)
    save_custom_model(model, None, str(tmp_path / "ckpt"))
    from safetensors.torch import load_file
    sd = load_file(str(tmp_path / "ckpt" / "model.safetensors"))
    assert torch.equal(sd["model.layers.0.self_attn.q_proj.weight"], layers[0].W_res)
    assert torch.equal(sd["model.layers.0.self_attn.q_proj.bias"], layers[0].bias)
    # adapters are restored afterwards
    from hdpissa_amd import CustomLinearLayer
    assert isinstance(model.model.layers[0].self_attn.q_proj, CustomLinearLayer)


def _trained_tiny(steps, seed=0):
    from hdpissa_amd import HDPissaStep, replace_with_custom_layer
    torch.manual_seed(seed)
    m = _tiny_model()
    layers = replace_with_custom_layer(m, ["q_proj", "o_proj", "down_proj"], 0, 1, 4, 4.0, ops=CpuOps())
    st = HDPissaStep(m, 1, 0, ops=CpuOps())
    g = torch.Generator().manual_seed(7)
    for t in range(steps):
        for L in layers:
            x = torch.randn(5, L.in_features, generator=g)
            gy = torch.randn(5, L.out_features, generator=g)
            L._probe_backward(x, gy)
        st.step(1e-2, t + 1)
    return m, layers, st


def test_resume_state_roundtrip(tmp_path):
    """save_hdpissa_state / load_hdpissa_state (the reference keeps m, v, t in
    memory only, hp:290-300): 2 steps + save + load into a fresh model + 1 step == 3 straight steps."""
    from hdpissa_amd import HDPissaStep, load_hdpissa_state, save_hdpissa_state
    full, full_layers, _ = _trained_tiny(3)
    part, part_layers, _ = _trained_tiny(2)
    path = str(tmp_path / "state.safetensors")
    save_hdpissa_state(part, path, t=2)
    fresh, fresh_layers, _ = _trained_tiny(0)
    t = load_hdpissa_state(fresh, path)
    assert t == 2
    for a, b in zip(part_layers, fresh_layers):
        assert torch.equal(a.W_res, b.W_res) and torch.equal(a.m_A, b.m_A) and torch.equal(a.v_B, b.v_B)
        assert torch.equal(a.A, b.A) and torch.equal(a.B, b.B)
    st = HDPissaStep(fresh, 1, 0, ops=CpuOps())
    g = torch.Generator().manual_seed(7)
    for _ in range(2):  # replay the generator to the third step's inputs
        for L in fresh_layers:
            torch.randn(5, L.in_features, generator=g)
            torch.randn(5, L.out_features, generator=g)
    for L in fresh_layers:
        L._probe_backward(torch.randn(5, L.in_features, generator=g), torch.randn(5, L.out_features, generator=g))
    st.step(1e-2, t + 1)
    for a, b in zip(full_layers, fresh_layers):
        assert torch.equal(a.W_res, b.W_res)
        assert torch.equal(a.m_B, b.m_B)


def test_resume_state_rejects_other_layout(tmp_path):
    from hdpissa_amd import load_hdpissa_state, replace_with_custom_layer, save_hdpissa_state
    m, _, _ = _trained_tiny(1)
    path = str(tmp_path / "s.safetensors")
    save_hdpissa_state(m, path, t=1)
    other = _tiny_model()
    replace_with_custom_layer(other, ["q_proj", "down_proj"], 0, 1, 4, 4.0, ops=CpuOps())
    with pytest.raises(ValueError, match="match"):
        load_hdpissa_state(other, path)


def test_resume_state_residual_mode(tmp_path):
    """Residual mode in the resume file: a residual-mode state loads only into a residual-mode model
    (same W_res, different effective weight otherwise), and the loaded model's forward and merged
    weights use the RESTORED factors (a fresh model's factors are overwritten by the load)."""
    from hdpissa_amd import load_hdpissa_state, replace_with_custom_layer, save_hdpissa_state

    def build(seed, residual):
        torch.manual_seed(seed)
        m = _tiny_model()
        layers = replace_with_custom_layer(m, ["q_proj", "down_proj"], 0, 1, 4, 4.0, ops=CpuOps(), residual=residual)
        return m, layers

    src, src_layers = build(0, True)
    with torch.no_grad():
        src_layers[0].W_res.add_(1e-3)
    path = str(tmp_path / "res.safetensors")
    save_hdpissa_state(src, path, t=5)
    plain, _ = build(0, False)
    with pytest.raises(ValueError, match="residual"):
        load_hdpissa_state(plain, path)
    dst, dst_layers = build(0, True)
    from hdpissa_amd.layer import _bind_residual_factors
    with torch.no_grad():  # other factors before the load (as a differently initialised run would have)
        dst_layers[0]._arena.fac_all.mul_(1.5)
        for L in dst_layers:
            _bind_residual_factors(L)
    assert not torch.equal(dst_layers[0].A, src_layers[0].A)
    assert load_hdpissa_state(dst, path) == 5
    x = torch.randn(3, 5, 32)
    y_src = src.model.layers[0].self_attn.q_proj(x)
    y_dst = dst.model.layers[0].self_attn.q_proj(x)
    assert torch.equal(y_src, y_dst)
    for a, b in zip(src_layers, dst_layers):
        assert torch.equal(a.merge_weights(), b.merge_weights())


def test_export_merged_safetensors(tmp_path):
    from safetensors.torch import load_file
    from hdpissa_amd import custom_layers, export_merged_safetensors
    m, layers, _ = _trained_tiny(2)
    path = str(tmp_path / "merged.safetensors")
    export_merged_safetensors(m, path)
    got = load_file(path)
    names = [n for n, _ in custom_layers(m)]
    assert sorted(got) == sorted(f"{n}.weight" for n in names)
    for n, L in custom_layers(m):
        assert torch.equal(got[f"{n}.weight"], L.W_res)   # the merged weight IS W_res (hp:142-144)


def test_pissa_residual_mode_cpu():
    """Opt-in PiSSA-residual mode (north star (1)): W_res = W - sum_i B_i A_i (all ranks' slices),
    forward and merged weight unchanged, and after a step the effective weight equals the default
    mode's W_res."""
    from hdpissa_amd import HDPissaStep, replace_with_custom_layer
    outs = {}
    for residual in (False, True):
        torch.manual_seed(3)
        m = _tiny_model()
        W0 = {n: mod.weight.detach().clone() for n, mod in m.named_modules() if isinstance(mod, nn.Linear)}
        layers = replace_with_custom_layer(m, ["q_proj", "down_proj"], 1, 2, 4, 4.0, ops=CpuOps(), residual=residual)
        x = torch.randn(3, 5, 32)
        y = m.model.layers[0].self_attn.q_proj(x)
        if residual:
            for L in layers:
                arena = L._arena
                i = arena.layers.index(L)
                A = [arena.views(arena.fac_all[d], i)[0].numpy() for d in range(2)]
                B = [arena.views(arena.fac_all[d], i)[1].numpy() for d in range(2)]
                ref = O.pissa_residual(W0[L.name].numpy(), A, B)
                assert rel_err(L.W_res.numpy(), ref) < 1e-6
                assert rel_err(L.merge_weights().numpy(), W0[L.name].numpy()) < 1e-6
        st = HDPissaStep(m, 2, 1, ops=CpuOps(), comm=_LoopbackComm(2))
        g = torch.Generator().manual_seed(11)
        for L in layers:
            L._probe_backward(torch.randn(6, L.in_features, generator=g), torch.randn(6, L.out_features, generator=g))
        st.step(1e-2, 1)
        outs[residual] = (y.detach(), [L.merge_weights() for L in layers])
    assert rel_err(outs[True][0].numpy(), outs[False][0].numpy()) < 1e-6
    for a, b in zip(outs[True][1], outs[False][1]):
        assert rel_err(a.numpy(), b.numpy()) < 1e-6


class _LoopbackComm:
    """Single-process stand-in for a 2-rank exchange: every rank's delta equals this rank's."""
    name = "loopback"

    def __init__(self, world_size):
        self.world_size = world_size

    def allgather(self, send, recv):
        recv.view(self.world_size, -1).copy_(send.reshape(1, -1).expand(self.world_size, -1))

    def allreduce_sum(self, buf):
        buf.mul_(self.world_size)

    def broadcast(self, t, root):
        pass


def test_comm_falls_back_to_torch_distributed(monkeypatch, capsys):
    """make_comm on a HIP device: if the library's RCCL communicator cannot be created, the step's
    collectives go through torch.distributed (RCCL on the GPU, not a host path), reported on stderr."""
    import torch

    from hdpissa_amd import comm as C

    class Boom:
        def __init__(self, *a, **k):
            raise RuntimeError("ncclCommInitRank failed: test")

    monkeypatch.setattr(C, "RcclComm", Boom)
    monkeypatch.delenv("HDP_COMM", raising=False)
    c = C.make_comm(1, 2, torch.device("cuda", 0))
    assert isinstance(c, C.TorchComm) and c.rank == 1 and c.world_size == 2
    assert "using torch.distributed collectives" in capsys.readouterr().err
    assert isinstance(C.make_comm(0, 1, torch.device("cuda", 0)), C.LocalComm)
