"""End-to-end training throughput: a real HF LlamaForCausalLM / MistralForCausalLM
of a BASELINE config's shape (random init -- no checkpoints offline), every projection replaced by the
drop-in CustomLinearLayer, trained by HDPissaTrainer on synthetic instruction micro-batches
(batch 2, prompt U[32,256] + response U[32,256] tokens, prompt and padding labels -100, padding
to the longest sample), accumulation 64 // 8 = 8 micro-batches per optimizer step (run.sh).

  python tools/e2e_train.py [--model llama2-7b|mistral-7b|llama2-13b] [--layers N] [--steps 2] [--warmup 1]
                            [--dtype float32|bfloat16] [--ref]

Prints one JSON line: train tokens/s of the whole step (HF forward + backward through the base
model, the K2 probes, and the HD-PiSSA step), and the share of the step spent in the hot path.
--ref also times the reference's own layer (hp:136-140: the out x in product B A materialised,
the extra fp32 GEMMs in forward and backward) and its step block (hp:352-398) in torch on the
same GPU, same model and batches.  Measurement tool: not part of the package.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hd-pissa_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402
import torch.nn.functional as F  # noqa: E402

TARGETS = ["q_proj", "o_proj", "k_proj", "v_proj", "gate_proj", "up_proj", "down_proj"]
# BASELINE.json configs: architecture, default dtype, r per GPU, alpha (alpha = r for r > 16:
# the reference's alpha // r (hp:103) with run.sh's alpha 16 would train nothing)
MODELS = {
    "llama2-7b": dict(cls="LlamaConfig", hidden=4096, inter=11008, layers=32, heads=32, kv_heads=32, vocab=32000,
                      dtype="float32", r=16, alpha=16.0),
    "mistral-7b": dict(cls="MistralConfig", hidden=4096, inter=14336, layers=32, heads=32, kv_heads=8, vocab=32000,
                       dtype="bfloat16", r=64, alpha=64.0),
    "llama2-13b": dict(cls="LlamaConfig", hidden=5120, inter=13824, layers=40, heads=40, kv_heads=40, vocab=32000,
                       dtype="bfloat16", r=128, alpha=128.0),
}


def batches(n, batch, vocab, seed, max_len=512):
    g = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        lp = g.integers(32, 257, batch)
        lr = g.integers(32, 257, batch)
        lens = np.minimum(lp + lr, max_len)
        L = int(lens.max())
        ids = torch.full((batch, L), 2, dtype=torch.long)   # pad = eos
        lab = torch.full((batch, L), -100, dtype=torch.long)
        for b in range(batch):
            row = torch.from_numpy(g.integers(3, vocab, int(lens[b])))
            ids[b, :lens[b]] = row
            lab[b, min(lp[b], lens[b]):lens[b]] = row[min(lp[b], lens[b]):]
        out.append(dict(input_ids=ids, labels=lab, attention_mask=ids.ne(2), tokens=int(lens.sum())))
    return out


class RefLayer(nn.Module):
    """The reference's CustomLinearLayer forward (hp:136-140) on given factors: the adapter term
    materialises M = B A * 1e-16 * alpha (out x in) and runs a second fp32 GEMM; autograd then
    forms dM = G^T x and the factor grads through it.  Timing baseline only."""

    def __init__(self, W, bias, A, B, alpha):
        super().__init__()
        self.register_buffer("W_res", W)
        self.bias = bias
        self.A = nn.Parameter(A.clone())
        self.B = nn.Parameter(B.clone())
        self.alpha = alpha
        self.m = [torch.zeros_like(A), torch.zeros_like(A), torch.zeros_like(B), torch.zeros_like(B)]

    def forward(self, x):
        x32 = x.float()
        M = (self.B @ self.A) * 1e-16 * self.alpha
        return F.linear(x, self.W_res, self.bias) + F.linear(x32, M).to(x.dtype)


def ref_step(model, lr, t, b1=0.9, b2=0.999, eps=1e-8):
    """hp:352-398 at world size 1 in torch (the all_gathers are identities)."""
    with torch.no_grad():
        for L in model.modules():
            if not isinstance(L, RefLayer):
                continue
            gA, gB = L.A.grad * 1e16, L.B.grad * 1e16
            L.m[0] = b1 * L.m[0] + (1 - b1) * gA
            L.m[1] = b2 * L.m[1] + (1 - b2) * gA ** 2
            L.m[2] = b1 * L.m[2] + (1 - b1) * gB
            L.m[3] = b2 * L.m[3] + (1 - b2) * gB ** 2
            dA = lr * (L.m[0] / (1 - b1 ** t)) / (torch.sqrt(L.m[1] / (1 - b2 ** t)) + eps)
            dB = lr * (L.m[2] / (1 - b1 ** t)) / (torch.sqrt(L.m[3] / (1 - b2 ** t)) + eps)
            dW = torch.zeros_like(L.W_res)
            dW -= dB @ L.A + L.B @ dA - dB @ dA
            L.W_res += dW.to(L.W_res.dtype)
            L.A.grad = None
            L.B.grad = None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=None, help="default: the config's own")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--micro", type=int, default=8)
    ap.add_argument("--model", default="llama2-7b", choices=sorted(MODELS))
    ap.add_argument("--dtype", default=None, choices=["float32", "bfloat16"], help="default: the config's own")
    ap.add_argument("--ref", action="store_true")
    args = ap.parse_args()
    import transformers
    from hdpissa_amd import HDPissaTrainer, custom_layers, get_parent_module, replace_with_custom_layer
    from hdpissa_amd.layer import CustomLinearLayer

    dev = torch.device("cuda:0")
    mc = MODELS[args.model]
    args.dtype = args.dtype or mc["dtype"]
    args.layers = args.layers or mc["layers"]
    dt = getattr(torch, args.dtype)
    cfg = getattr(transformers, mc["cls"])(hidden_size=mc["hidden"], intermediate_size=mc["inter"],
                                           num_hidden_layers=args.layers, num_attention_heads=mc["heads"],
                                           num_key_value_heads=mc["kv_heads"], vocab_size=mc["vocab"],
                                           max_position_embeddings=4096, attn_implementation="sdpa")
    t0 = time.time()
    torch.manual_seed(0)
    with torch.device(dev):
        model = getattr(transformers, mc["cls"].replace("Config", "ForCausalLM"))(cfg).to(dt)
    for p in model.parameters():
        p.requires_grad = False
    t_model = time.time() - t0
    t0 = time.time()
    layers = replace_with_custom_layer(model, TARGETS, 0, 1, mc["r"], mc["alpha"])
    torch.cuda.synchronize()
    t_init = time.time() - t0
    bs = batches((args.warmup + args.steps) * args.micro, 2, cfg.vocab_size, 42)
    tr = HDPissaTrainer(model, 1, 0, 2e-5, 1000, args.micro, warmup_ratio=0.03, loss_sync="step")

    def run(step_fn, micro_fn, n_steps, it):
        tok = 0
        for _ in range(n_steps):
            for _ in range(args.micro):
                b = next(it)
                tok += b["tokens"]
                micro_fn(b)
            step_fn()
        return tok

    it = iter(bs)
    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    hot = [0.0]

    def micro_ours(b):
        tr.micro_step(b)

    run(lambda: None, micro_ours, args.warmup, it)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tok = run(lambda: None, micro_ours, args.steps, it)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    res = dict(metric=f"end-to-end train tokens/s, HF {mc['cls'].replace('Config', 'ForCausalLM')} ({args.model} shape" +
               (f", {args.layers} layers" if args.layers != mc["layers"] else "") + f", {args.dtype}) + HD-PiSSA r{mc['r']}, 1 GPU",
               model=args.model, dtype=args.dtype, r=mc["r"],
               value=round(tok / el, 1), unit="tokens/s", steps=args.steps, micro_batches_per_step=args.micro,
               ms_per_step=round(1e3 * el / args.steps, 1), model_build_s=round(t_model, 1), svd_init_s=round(t_init, 1),
               loss=tr.loss_list[-args.steps:])
    if args.ref:
        # the reference's layer + step on the same model, factors and batches
        for name, L in custom_layers(model):
            R = RefLayer(L.W_res, L.bias, L.A.detach(), L.B.detach(), L.alpha)
            setattr(get_parent_module(model, name), name.split(".")[-1], R)
        del layers, tr
        torch.cuda.empty_cache()
        state = dict(t=0)

        def micro_ref(b):
            out = model(input_ids=b["input_ids"].to(dev), attention_mask=b["attention_mask"].to(dev),
                        labels=b["labels"].to(dev))
            (out.loss / args.micro).backward()

        def step_ref():
            state["t"] += 1
            ref_step(model, 2e-5, state["t"])

        it = iter(bs)
        run(step_ref, micro_ref, args.warmup, it)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tok_r = run(step_ref, micro_ref, args.steps, it)
        torch.cuda.synchronize()
        el_r = time.perf_counter() - t0
        res["reference_layer_torch"] = dict(value=round(tok_r / el_r, 1), ms_per_step=round(1e3 * el_r / args.steps, 1))
        res["speedup_vs_reference_layer"] = round((tok / el) / (tok_r / el_r), 2)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
