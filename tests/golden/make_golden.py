"""Generate golden vectors from the reference implementation (build container only).

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

It imports ``/root/reference/hd_pissa.py`` (read-only, never copied) and runs the
reference's own code on small seeded inputs:

* ``CustomLinearLayer.__init__`` (hp:96-134)       -> svd_*.npz   (A, B per rank, S)
* ``CustomLinearLayer.forward`` + autograd (hp:136-140) -> probe_*.npz (y, A.grad, B.grad
  after each of 3 accumulated micro-steps)
* the literal optimizer-step block ``hp:352-398`` (extracted from
  ``inspect.getsource(main)`` with ``ast`` and exec'd unchanged in each of Wn gloo CPU
  processes)                                      -> step_*.npz   (grads, Adam state,
  W_res after each of 3 steps, every rank)
* the literal LR-schedule block ``hp:338-344``    -> lr_schedule.npz

Only data (inputs and outputs) is written; no reference source is stored.
"""
from __future__ import annotations

import ast
import inspect
import math
import os
import socket
import sys
import tempfile
import textwrap

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def _ref():
    sys.dont_write_bytecode = True
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import hd_pissa  # noqa: E402
    return hd_pissa


def _main_block(kind: str) -> str:
    """Source text of a block inside ``hd_pissa.main``: 'step' = the
    ``with torch.no_grad():`` update block (hp:352-398); 'lr' = the
    ``if t < warmup_steps:`` schedule block (hp:338-344); 'loop' = the micro-step loop
    ``for i, batch in enumerate(dataloader):`` (hp:320-400)."""
    hp = _ref()
    src = textwrap.dedent(inspect.getsource(hp.main))
    tree = ast.parse(src)
    for node in ast.walk(tree):
        if kind == "step" and isinstance(node, ast.With):
            call = node.items[0].context_expr
            if isinstance(call, ast.Call) and ast.unparse(call.func) == "torch.no_grad":
                return ast.unparse(node)
        if kind == "lr" and isinstance(node, ast.If) and ast.unparse(node.test) == "t < warmup_steps":
            return ast.unparse(node)
        if kind == "loop" and isinstance(node, ast.For) and ast.unparse(node.target) in ("(i, batch)", "i, batch"):
            return ast.unparse(node)
    raise RuntimeError(f"block {kind} not found")


def spectrum_matrix(out, inn, seed, decay=0.9):
    """W = Q1 diag(s) Q2^T with well-separated singular values (s_k = decay^k)."""
    g = torch.Generator().manual_seed(seed)
    k = min(out, inn)
    q1, _ = torch.linalg.qr(torch.randn(out, k, generator=g, dtype=torch.float64))
    q2, _ = torch.linalg.qr(torch.randn(inn, k, generator=g, dtype=torch.float64))
    s = decay ** torch.arange(k, dtype=torch.float64)
    return (q1 * s) @ q2.T


def gaussian_matrix(out, inn, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(out, inn, generator=g, dtype=torch.float64) * 0.02


def make_linear(W, bias_seed=None, dtype=torch.float32):
    lin = torch.nn.Linear(W.shape[1], W.shape[0], bias=bias_seed is not None)
    with torch.no_grad():
        lin.weight.copy_(W.to(torch.float32))
        if bias_seed is not None:
            g = torch.Generator().manual_seed(bias_seed)
            lin.bias.copy_(torch.randn(W.shape[0], generator=g) * 0.1)
    return lin.to(dtype)


# ----------------------------------------------------------------------------
def gen_svd():
    hp = _ref()
    cases = {
        "tall_spec": spectrum_matrix(64, 48, 1),
        "wide_spec": spectrum_matrix(40, 72, 2),
        "sq_gauss": gaussian_matrix(56, 56, 3),
    }
    for name, W in cases.items():
        for dt_name, dt in (("f32", torch.float32), ("bf16", torch.bfloat16)):
            lin = make_linear(W, dtype=dt)
            rec = {"W": lin.weight.detach().float().numpy()}
            Wf = lin.weight.detach().float()
            rec["S"] = torch.linalg.svdvals(Wf.double()).numpy()
            for r in (4, 8):
                for wn in (1, 2, 4):
                    if r * wn > min(W.shape):
                        continue
                    for d in range(wn):
                        layer = hp.CustomLinearLayer(lin, "q_proj", d, wn, ranks_per_gpu=r, alpha=16.0)
                        assert torch.equal(layer.W_res, lin.weight.data), "W_res must be W (hp:129)"
                        assert layer.W_res.dtype == dt
                        rec[f"A_r{r}_w{wn}_d{d}"] = layer.A.detach().numpy()
                        rec[f"B_r{r}_w{wn}_d{d}"] = layer.B.detach().numpy()
            np.savez_compressed(os.path.join(OUT, f"svd_{name}_{dt_name}.npz"), **rec)


def gen_probe():
    hp = _ref()
    cases = [
        # name, out, in, r, wn, d, alpha, dtype, bias
        ("f32_bias", 64, 48, 4, 2, 1, 16.0, torch.float32, True),
        ("f32_wide", 40, 72, 8, 2, 0, 16.0, torch.float32, False),
        ("bf16_bias", 64, 48, 4, 2, 0, 16.0, torch.bfloat16, True),
        ("alpha_floor_zero", 64, 48, 4, 1, 0, 3.0, torch.float32, False),   # 3 // 4 = 0
        ("alpha_floor_frac", 64, 48, 4, 1, 0, 7.0, torch.float32, False),   # 7 // 4 = 1
    ]
    for i, (name, out, inn, r, wn, d, alpha, dt, bias) in enumerate(cases):
        W = spectrum_matrix(out, inn, 10 + i)
        lin = make_linear(W, bias_seed=(20 + i) if bias else None, dtype=dt)
        layer = hp.CustomLinearLayer(lin, "q_proj", d, wn, ranks_per_gpu=r, alpha=alpha)
        rec = {"W": lin.weight.detach().float().numpy(), "A": layer.A.detach().numpy(),
               "B": layer.B.detach().numpy(), "alpha_eff": np.float64(layer.alpha),
               "alpha": np.float64(alpha), "r": np.int64(r)}
        if bias:
            rec["bias"] = lin.bias.detach().float().numpy()
        g = torch.Generator().manual_seed(100 + i)
        for ms in range(3):
            x = torch.randn(2, 3, inn, generator=g).to(dt)
            G = torch.randn(2, 3, out, generator=g).to(dt)
            y = layer(x)
            y.backward(G)
            base = torch.nn.functional.linear(x, layer.W_res, layer.bias)
            rec[f"x{ms}"] = x.float().numpy()
            rec[f"G{ms}"] = G.float().numpy()
            rec[f"y{ms}"] = y.detach().float().numpy()
            rec[f"y_equals_base{ms}"] = np.bool_(torch.equal(y, base))
            rec[f"gA{ms}"] = layer.A.grad.detach().clone().numpy()
            rec[f"gB{ms}"] = layer.B.grad.detach().clone().numpy()
        np.savez_compressed(os.path.join(OUT, f"probe_{name}.npz"), **rec)


# ----------------------------------------------------------------------------
STEP_CASES = [
    # name, modules [(name, out, in, bias)], r, alpha, dtype, lrs per step
    ("f32_tall", [("layers.0.q_proj", 64, 48, True)], 4, 16.0, torch.float32, [1e-2, 5e-3, 2e-3]),
    ("f32_wide", [("layers.0.down_proj", 40, 72, False)], 4, 16.0, torch.float32, [1e-2, 5e-3, 2e-3]),
    ("bf16_tall", [("layers.0.q_proj", 64, 48, True)], 4, 16.0, torch.bfloat16, [1e-2, 5e-3, 2e-3]),
    ("f32_two", [("layers.0.q_proj", 48, 48, False), ("layers.1.up_proj", 64, 32, False)], 4, 8.0,
     torch.float32, [3e-3, 3e-3, 3e-3]),
]


class _Container(torch.nn.Module):
    def __init__(self, specs, dtype):
        super().__init__()
        self.layers = torch.nn.ModuleList()
        for j, (name, out, inn, bias) in enumerate(specs):
            idx = int(name.split(".")[1])
            while len(self.layers) <= idx:
                self.layers.append(torch.nn.Module())
            W = spectrum_matrix(out, inn, 300 + j, decay=0.93)
            setattr(self.layers[idx], name.split(".")[-1], make_linear(W, bias_seed=(400 + j) if bias else None, dtype=dtype))


def _step_worker(rank, wn, port, case_idx, tmpdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=wn)
    torch.manual_seed(0)
    hp = _ref()
    name, specs, r, alpha, dt, lrs = STEP_CASES[case_idx]
    model = _Container(specs, dt)
    for p in model.parameters():
        p.requires_grad = False
    targets = [s[0].split(".")[-1] for s in specs]
    hp.replace_with_custom_layer(model, targets, rank, wn, ranks_per_gpu=r, alpha=alpha)
    layers = [(n, m) for n, m in model.named_modules() if isinstance(m, hp.CustomLinearLayer)]
    for _, layer in layers:                                   # hp:290-295 (on CPU)
        layer.m_A = torch.zeros_like(layer.A.data)
        layer.v_A = torch.zeros_like(layer.A.data)
        layer.m_B = torch.zeros_like(layer.B.data)
        layer.v_B = torch.zeros_like(layer.B.data)
    block = compile(_main_block("step"), "<hp:352-398>", "exec")
    rec = {}
    for j, (n, layer) in enumerate(layers):
        rec[f"{j}.A"] = layer.A.detach().numpy()
        rec[f"{j}.B"] = layer.B.detach().numpy()
        rec[f"{j}.W0"] = layer.W_res.detach().float().clone().numpy()
        rec[f"{j}.alpha_eff"] = np.float64(layer.alpha)
    t = 0
    g = torch.Generator().manual_seed(1000 + 17 * rank + case_idx)
    for step, lr in enumerate(lrs):
        for j, (n, layer) in enumerate(layers):
            for ms in range(2):                                  # 2 accumulated micro-steps
                x = torch.randn(2, 3, layer.in_features, generator=g).to(dt)
                G = torch.randn(2, 3, layer.out_features, generator=g).to(dt)
                layer(x).backward(G)
            rec[f"s{step}.{j}.gA"] = layer.A.grad.detach().clone().numpy()
            rec[f"s{step}.{j}.gB"] = layer.B.grad.detach().clone().numpy()
            for k in ("m_A", "v_A", "m_B", "v_B"):
                rec[f"s{step}.{j}.{k}_in"] = getattr(layer, k).detach().clone().numpy()
        t += 1                                                   # hp:350
        ns = {"torch": torch, "dist": dist, "model": model, "CustomLinearLayer": hp.CustomLinearLayer,
              "beta1": 0.9, "beta2": 0.999, "epsilon": 1e-08, "t": t, "lr": lr, "world_size": wn}
        exec(block, ns)
        for j, (n, layer) in enumerate(layers):
            rec[f"s{step}.{j}.W"] = layer.W_res.detach().float().clone().numpy()
            for k in ("m_A", "v_A", "m_B", "v_B"):
                rec[f"s{step}.{j}.{k}_out"] = getattr(layer, k).detach().clone().numpy()
            assert layer.A.grad is None and layer.B.grad is None
        if len(layers) == 1:
            rec[f"s{step}.0.delta_A"] = ns["delta_A"].numpy()
            rec[f"s{step}.0.delta_B"] = ns["delta_B"].numpy()
            rec[f"s{step}.0.dW"] = ns["delta_W_res"].float().clone().numpy()
        rec[f"s{step}.t"] = np.int64(t)
        rec[f"s{step}.lr"] = np.float64(lr)
    np.savez(os.path.join(tmpdir, f"rank{rank}.npz"), **rec)
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def gen_step(wns=(1, 2, 4), names=None):
    for ci, case in enumerate(STEP_CASES):
        if names is not None and case[0] not in names:
            continue
        for wn in wns:
            with tempfile.TemporaryDirectory() as td:
                mp.spawn(_step_worker, args=(wn, _free_port(), ci, td), nprocs=wn, join=True)
                rec = {"world_size": np.int64(wn), "r": np.int64(case[2]), "alpha": np.float64(case[3]),
                       "dtype": np.str_("bfloat16" if case[4] == torch.bfloat16 else "float32"),
                       "n_modules": np.int64(len(case[1])), "n_steps": np.int64(len(case[5]))}
                for rk in range(wn):
                    with np.load(os.path.join(td, f"rank{rk}.npz")) as z:
                        for k in z.files:
                            rec[f"r{rk}.{k}"] = z[k]
            np.savez_compressed(os.path.join(OUT, f"step_{case[0]}_w{wn}.npz"), **rec)


def gen_step8():
    """World size 8 (the BASELINE node) for the 64 x 48, r = 4 cases: r * 8 = 32 <= 48 triplets."""
    torch.set_num_threads(1)
    gen_step(wns=(8,), names=("f32_tall", "bf16_tall"))


def gen_lr():
    block = compile(_main_block("lr"), "<hp:338-344>", "exec")
    rows = []
    for schedule in ("cosine", "linear"):
        for warmup_steps, total_steps in ((0, 10), (3, 10), (1, 5)):
            for t in range(total_steps + 1):
                ns = {"math": __import__("math"), "t": t, "warmup_steps": warmup_steps, "initial_lr": 2e-5,
                      "total_steps": total_steps, "schedule": schedule}
                exec(block, ns)
                rows.append((1 if schedule == "cosine" else 0, warmup_steps, total_steps, t, ns["lr"]))
    np.savez_compressed(os.path.join(OUT, "lr_schedule.npz"), rows=np.array(rows, dtype=np.float64))


# ----------------------------------------------------------------------------
# data path (hp:158-210) with a deterministic stub tokenizer (tests/helpers.py)
def _helpers():
    here = os.path.dirname(OUT)
    if here not in sys.path:
        sys.path.insert(0, here)
    import helpers
    return helpers


def _ragged(prefix, rows, rec):
    rec[f"{prefix}_flat"] = np.concatenate([np.asarray(r, np.int64) for r in rows]) if rows else np.zeros(0, np.int64)
    rec[f"{prefix}_len"] = np.array([len(r) for r in rows], np.int64)


def gen_data():
    hp = _ref()
    H = _helpers()
    tok = H.StubTokenizer(model_max_length=200)
    ex = H.synthetic_instructions(20, 7)
    out = hp.train_tokenize_function(ex, tok, "query", "response")           # hp:206-210 -> 171-184
    rec = {"query": np.array(ex["query"]), "response": np.array(ex["response"]),
           "model_max_length": np.int64(200)}
    _ragged("input_ids", [list(x) for x in out["input_ids"]], rec)
    _ragged("labels", [list(x) for x in out["labels"]], rec)
    inst = [{"input_ids": out["input_ids"][i], "labels": out["labels"][i]} for i in range(4)]
    coll = hp.DataCollatorForSupervisedDataset(tokenizer=tok)(inst)         # hp:186-204
    for k, v in coll.items():
        rec[f"collated_{k}"] = v.numpy()
    # the reference's dataset pipeline (hp:243-261) on an in-memory dataset: map, filter, shuffle(42)
    import datasets
    raw = datasets.Dataset.from_dict(ex)
    ds = raw.map(hp.train_tokenize_function, batched=True, batch_size=3000, remove_columns=raw.column_names,
                 fn_kwargs={"tokenizer": tok, "query": "query", "response": "response"})
    ds = ds.filter(lambda e: not all(label == -100 for label in e["labels"])).shuffle(seed=42)
    _ragged("pipeline_input_ids", [list(r) for r in ds["input_ids"]], rec)
    np.savez_compressed(os.path.join(OUT, "data_path.npz"), **rec)


# ----------------------------------------------------------------------------
# plumbing trajectory: a tiny Qwen2 through the reference's own
# replace_with_custom_layer (hp:150-156) and its literal micro-step loop (hp:320-400, which
# contains the schedule and the update block hp:352-398), under gloo
TRAJ = dict(r=8, alpha=8.0, lr=2e-3, steps=5, accumulation=2, batch=2)


class _HostTensor(torch.Tensor):
    """Batch tensors whose .cuda(rank, non_blocking=True) (hp:321-323) stays on the host."""

    def cuda(self, *a, **k):
        return self.as_subclass(torch.Tensor)


def _traj_batches(rank, n, H, batch=None):
    batch = TRAJ["batch"] if batch is None else batch
    tok = H.StubTokenizer(model_max_length=200)
    hp = _ref()
    ex = H.synthetic_instructions(4 * n * batch, 500 + rank)
    out = hp.train_tokenize_function(ex, tok, "query", "response")
    keep = [i for i in range(len(out["labels"])) if not all(l == -100 for l in out["labels"][i])]
    coll = hp.DataCollatorForSupervisedDataset(tokenizer=tok)
    bs = []
    for b in range(n):
        idx = keep[b * batch:(b + 1) * batch]
        bs.append(coll([{"input_ids": out["input_ids"][i], "labels": out["labels"][i]} for i in idx]))
    return bs


def _traj_worker(rank, wn, port, tmpdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=wn)
    torch.set_num_threads(2)
    hp = _ref()
    H = _helpers()
    from transformers import Qwen2Config, Qwen2ForCausalLM
    torch.manual_seed(1234)
    model = Qwen2ForCausalLM(Qwen2Config(**H.QWEN_TINY, attn_implementation="eager")).float()
    rec = {}
    if rank == 0:
        for k, v in model.state_dict().items():
            rec[f"state.{k}"] = v.detach().clone().numpy()
    for p in model.parameters():
        p.requires_grad = False
    hp.replace_with_custom_layer(model, H.QWEN_TARGETS, rank, wn, ranks_per_gpu=TRAJ["r"], alpha=TRAJ["alpha"])
    layers = [(n, m) for n, m in model.named_modules() if isinstance(m, hp.CustomLinearLayer)]
    for j, (n, layer) in enumerate(layers):                                   # hp:290-295
        layer.m_A = torch.zeros_like(layer.A.data)
        layer.v_A = torch.zeros_like(layer.A.data)
        layer.m_B = torch.zeros_like(layer.B.data)
        layer.v_B = torch.zeros_like(layer.B.data)
        rec[f"mod{j}.name"] = np.str_(n)
        rec[f"mod{j}.A"] = layer.A.detach().numpy()
        rec[f"mod{j}.B"] = layer.B.detach().numpy()
    acc, steps = TRAJ["accumulation"], TRAJ["steps"]
    batches = _traj_batches(rank, steps * acc, H)
    for i, b in enumerate(batches):
        for k, v in b.items():
            rec[f"mb{i}.{k}"] = v.numpy()

    def loader():
        for i, b in enumerate(batches):
            if i and i % acc == 0:
                s = i // acc - 1
                for j, (_, layer) in enumerate(layers):
                    W = layer.W_res.detach().double()
                    rec[f"s{s}.{j}.wsum"] = np.float64(W.sum())
                    rec[f"s{s}.{j}.wsq"] = np.float64((W * W).sum())
            yield {k: v.as_subclass(_HostTensor) for k, v in b.items()}
    outdir = os.path.join(tmpdir, "out")
    ns = {"torch": torch, "dist": dist, "math": math, "os": os, "model": model, "CustomLinearLayer": hp.CustomLinearLayer,
          "dataloader": loader(), "accumulation_steps": acc, "world_size": wn, "rank": rank, "beta1": 0.9,
          "beta2": 0.999, "epsilon": 1e-08, "t": 0, "warmup_steps": 0, "total_steps": steps, "schedule": "cosine",
          "initial_lr": TRAJ["lr"], "lr": TRAJ["lr"], "loss_list": [], "current_step": 1, "accumulated_loss": 0,
          "output_path": outdir}
    exec(compile(_main_block("loop"), "<hp:320-400>", "exec"), ns)
    s = steps - 1
    for j, (_, layer) in enumerate(layers):
        W = layer.W_res.detach().double()
        rec[f"s{s}.{j}.wsum"] = np.float64(W.sum())
        rec[f"s{s}.{j}.wsq"] = np.float64((W * W).sum())
        rec[f"final.{j}.W"] = layer.W_res.detach().float().numpy()
    rec["loss_list"] = np.array(ns["loss_list"], np.float64)
    np.savez(os.path.join(tmpdir, f"rank{rank}.npz"), **rec)
    dist.barrier()
    dist.destroy_process_group()


def gen_trajectory():
    H = _helpers()
    for wn in (1, 2):
        with tempfile.TemporaryDirectory() as td:
            mp.spawn(_traj_worker, args=(wn, _free_port(), td), nprocs=wn, join=True)
            rec = {"world_size": np.int64(wn), **{k: np.float64(v) if isinstance(v, float) else np.int64(v)
                                                 for k, v in TRAJ.items()},
                   "config": np.str_(repr(sorted(H.QWEN_TINY.items()))), "targets": np.array(H.QWEN_TARGETS)}
            for rk in range(wn):
                with np.load(os.path.join(td, f"rank{rk}.npz")) as z:
                    for k in z.files:
                        rec[k if k.startswith("state.") else f"r{rk}.{k}"] = z[k]
        np.savez_compressed(os.path.join(OUT, f"trajectory_qwen2_w{wn}.npz"), **rec)


# ----------------------------------------------------------------------------
# plumbing config P at its real shape (BASELINE configs[0]: Qwen2.5-0.5B fp32, r = 16 per rank,
# world size 2 under gloo): the Qwen2.5-0.5B architecture (24 layers, 168 targeted projections;
# random init from a recorded seed -- no checkpoint offline), the reference's own
# replace_with_custom_layer (hp:150-156: its full torch.svd of every module) and its literal
# micro-step loop hp:320-400.  The weights are too large for a fixture, so only checksums are
# kept: per step the loss and, per module, sum((W_s - W_0)^2) and sum((W_s - W_0) * R) with R a
# fixed +-1 pattern (update checksums: the update is ~1e-5 of W), plus sum(W_s^2).
PLUMB = dict(r=16, alpha=16.0, lr=2e-5, steps=20, accumulation=2, batch=2, seed=1234)


def plumb_sign_pattern(j, shape):
    """The +-1 pattern of module j's dproj checksum (regenerated identically by the test)."""
    g = torch.Generator().manual_seed(7919 * (j + 1))
    return torch.randint(0, 2, tuple(shape), generator=g, dtype=torch.int8).double() * 2 - 1


def _plumb_worker(rank, wn, port, tmpdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=wn)
    torch.set_num_threads(max(1, 8 // wn))
    hp = _ref()
    H = _helpers()
    from transformers import Qwen2Config, Qwen2ForCausalLM
    torch.manual_seed(PLUMB["seed"])
    model = Qwen2ForCausalLM(Qwen2Config(**H.QWEN_05B, attn_implementation="eager")).float()
    rec = {"init_check": np.array(H.model_checksums(model), np.float64)}
    for p in model.parameters():
        p.requires_grad = False
    hp.replace_with_custom_layer(model, H.QWEN_TARGETS, rank, wn, ranks_per_gpu=PLUMB["r"], alpha=PLUMB["alpha"])
    layers = [(n, m) for n, m in model.named_modules() if isinstance(m, hp.CustomLinearLayer)]
    W0 = []
    for j, (n, layer) in enumerate(layers):                                   # hp:290-295
        layer.m_A = torch.zeros_like(layer.A.data)
        layer.v_A = torch.zeros_like(layer.A.data)
        layer.m_B = torch.zeros_like(layer.B.data)
        layer.v_B = torch.zeros_like(layer.B.data)
        rec[f"mod{j}.name"] = np.str_(n)
        W0.append(layer.W_res.detach().double().clone())
    acc, steps = PLUMB["accumulation"], PLUMB["steps"]
    batches = _traj_batches(rank, steps * acc, H, PLUMB["batch"])
    for i, b in enumerate(batches):
        for k, v in b.items():
            rec[f"mb{i}.{k}"] = v.numpy()

    def check(s):
        for j, (_, layer) in enumerate(layers):
            W = layer.W_res.detach().double()
            D = W - W0[j]
            rec[f"s{s}.{j}.dsq"] = np.float64((D * D).sum())
            rec[f"s{s}.{j}.dproj"] = np.float64((D * plumb_sign_pattern(j, D.shape)).sum())
            rec[f"s{s}.{j}.wsq"] = np.float64((W * W).sum())

    def loader():
        for i, b in enumerate(batches):
            if i and i % acc == 0:
                check(i // acc - 1)
            yield {k: v.as_subclass(_HostTensor) for k, v in b.items()}
    outdir = os.path.join(tmpdir, "out")
    ns = {"torch": torch, "dist": dist, "math": math, "os": os, "model": model, "CustomLinearLayer": hp.CustomLinearLayer,
          "dataloader": loader(), "accumulation_steps": acc, "world_size": wn, "rank": rank, "beta1": 0.9,
          "beta2": 0.999, "epsilon": 1e-08, "t": 0, "warmup_steps": int(0.03 * steps), "total_steps": steps,
          "schedule": "cosine", "initial_lr": PLUMB["lr"], "lr": PLUMB["lr"], "loss_list": [], "current_step": 1,
          "accumulated_loss": 0, "output_path": outdir}
    exec(compile(_main_block("loop"), "<hp:320-400>", "exec"), ns)
    check(steps - 1)
    rec["loss_list"] = np.array(ns["loss_list"], np.float64)
    np.savez(os.path.join(tmpdir, f"rank{rank}.npz"), **rec)
    dist.barrier()
    dist.destroy_process_group()


def gen_plumbing():
    H = _helpers()
    for wn in (1, 2):
        with tempfile.TemporaryDirectory() as td:
            mp.spawn(_plumb_worker, args=(wn, _free_port(), td), nprocs=wn, join=True)
            rec = {"world_size": np.int64(wn), **{k: np.float64(v) if isinstance(v, float) else np.int64(v)
                                                 for k, v in PLUMB.items()},
                   "config": np.str_(repr(sorted(H.QWEN_05B.items()))), "targets": np.array(H.QWEN_TARGETS)}
            for rk in range(wn):
                with np.load(os.path.join(td, f"rank{rk}.npz")) as z:
                    nmod = sum(1 for k in z.files if k.startswith("mod") and k.endswith(".name"))
                    for q in ("dsq", "dproj", "wsq"):  # [steps][modules]
                        rec[f"r{rk}.{q}"] = np.array([[z[f"s{s}.{j}.{q}"] for j in range(nmod)]
                                                      for s in range(PLUMB["steps"])], np.float64)
                    rec[f"r{rk}.names"] = np.array([str(z[f"mod{j}.name"]) for j in range(nmod)])
                    for k in z.files:
                        if k.startswith("mb"):
                            rec[f"r{rk}.{k}"] = z[k].astype(np.int32)
                    rec[f"r{rk}.loss_list"] = z["loss_list"]
                    rec[f"r{rk}.init_check"] = z["init_check"]
        np.savez_compressed(os.path.join(OUT, f"plumbing_qwen05b_w{wn}.npz"), **rec)


if __name__ == "__main__":
    torch.set_num_threads(4)
    which = sys.argv[1:] or ["lr", "svd", "probe", "step", "data", "trajectory", "plumbing"]
    for name in which:
        globals()[f"gen_{name}"]()
    print("golden vectors written to", OUT, ":", which)
