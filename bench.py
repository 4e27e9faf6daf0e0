"""bench.py -- HD-PiSSA hot path on MI355X (one JSON line on rank 0).

A "step" is one pass of the hot path over one batch of synthetic instruction data, at the
reference's documented configuration (run.sh): batch 2 x max_length 512, accumulation
64 // 8 = 8 micro-batches per rank per optimizer step, r = 16 per GPU, alpha = 16, all seven
projections of every decoder layer targeted.  Per step, on every rank:

  8 x  adapter probe fwd/bwd (K2) for every targeted module on that micro-batch's activations
       X and output gradients G (synthetic, resident in HBM; a micro-batch is batch x longest-
       sample rows, padded like the reference's collator).  X is laid out as a decoder delivers
       it to autograd: q/k/v of a layer read ONE normed hidden state, gate/up ONE, o and down
       their own (hp:139 is called per projection with that shared tensor); G is per module
  1 x  optimizer step: Adam on the factor arena (K3) -> RCCL exchange -> fused delta-GEMM
       merge W_res += sum_i (B'_i A'_i - B_i A_i) (K4) [exchange=allreduce: K4 store ->
       all-reduce -> K5 merge]

value = non-padding tokens of all ranks' micro-batches / step time (max over ranks); per-GPU
work is fixed as N grows ("weak").  The base model's own linears / attention are not part of
this path and are not run.  Extras on the line: the dW aggregate+merge time per
step (the metric's second half), the live roofline of the dominant kernel, the reference
algorithm's CPU baseline, and the reference torch path on the same GPU.

  python bench.py [--gpus N --steps K --warmup W] [--workload llama2-7b|qproj|mistral-7b|
                  llama2-13b|qwen2.5-0.5b] [--exchange gather|allreduce]
  N > 1: python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N
         or plainly `python bench.py --gpus N`: without WORLD_SIZE in the environment the bench starts
         the N ranks itself (a torch.distributed.run child, before this process touches the GPU) and
         relays rank 0's JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
import zlib

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hd-pissa_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import torch.nn as nn  # noqa: E402

# hidden, intermediate, kv_dim, layers, model dtype, r, alpha
WORKLOADS = {
    "llama2-7b": dict(hidden=4096, inter=11008, kv=4096, layers=32, dtype="float32", r=16, alpha=16.0,
                      targets="q_proj o_proj k_proj v_proj gate_proj up_proj down_proj"),
    "qproj": dict(hidden=4096, inter=11008, kv=4096, layers=1, dtype="float32", r=16, alpha=16.0, targets="q_proj"),
    # alpha = r for the r=64 / r=128 configs: the reference's `alpha // ranks_per_gpu` (hp:103) with
    # run.sh's alpha 16 would be 0 there (zero probe grads, nothing trained)
    "mistral-7b": dict(hidden=4096, inter=14336, kv=1024, layers=32, dtype="bfloat16", r=64, alpha=64.0,
                       targets="q_proj o_proj k_proj v_proj gate_proj up_proj down_proj"),
    "llama2-13b": dict(hidden=5120, inter=13824, kv=5120, layers=40, dtype="bfloat16", r=128, alpha=128.0,
                       targets="q_proj o_proj k_proj v_proj gate_proj up_proj down_proj"),
    "qwen2.5-0.5b": dict(hidden=896, inter=4864, kv=128, layers=24, dtype="float32", r=16, alpha=16.0,
                         targets="q_proj o_proj k_proj v_proj gate_proj up_proj down_proj"),
    # the CPU harness's workload (tests/test_bench_dist.py): the orchestration at toy size
    "tiny-test": dict(hidden=64, inter=96, kv=32, layers=2, dtype="float32", r=4, alpha=4.0,
                      targets="q_proj o_proj k_proj v_proj gate_proj up_proj down_proj"),
    # the same with a bf16 model: the rank-ordered bf16 all-reduce leg (all-to-all, fold, all-gather)
    "tiny-test-bf16": dict(hidden=64, inter=96, kv=32, layers=2, dtype="bfloat16", r=4, alpha=4.0,
                           targets="q_proj o_proj k_proj v_proj gate_proj up_proj down_proj"),
}
PEAK_HBM_GBS = 8000.0       # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
# MFMA ceilings, in f32-EQUIVALENT TFLOP/s (the flops of the f32 product each kernel computes), by
# the math the kernel runs (MI355X_MICROARCH.md: f32 MFMA 157.3 TF = the vector rate; bf16/f16
# dense 2.5 PF on 16x16x32 / 32x32x16; tools/mfma_rate.hip measures the 16x16x16 "_1k" form):
PEAK_MFMA_TFS = {
    "f32": 157.3,          # v_mfma_f32_16x16x4_f32 / 32x32x2_f32 (K2 float32, K4 f32)
    "x3": 2500.0 / 6,      # K4 bf16x3: six 32x32x16 bf16 products per f32 product
    "h2": 2500.0 / 3,      # K4 H2: three 32x32x16 f16 products per f32 product
    "bf16x3": 2500.0 / 3,  # K2 bf16 activations: three 16x16x16 bf16 products per f32 product
}
PEAK_F32_MFMA_TFS = PEAK_MFMA_TFS["f32"]
TRAFFIC_BOUND_BPS = 4.5e12  # measured HBM traffic rate above which a kernel is labelled HBM-bound


class _Blk(nn.Module):
    pass


def build_model(wl, device, seed=0):
    """LLaMA-style module tree with random-init nn.Linear weights (identical on every rank,
    like a loaded checkpoint).  Only the targeted projections are materialised."""
    H, I, KV = wl["hidden"], wl["inter"], wl["kv"]
    dt = getattr(torch, wl["dtype"])
    shapes = {"q_proj": (H, H), "k_proj": (KV, H), "v_proj": (KV, H), "o_proj": (H, H),
              "gate_proj": (I, H), "up_proj": (I, H), "down_proj": (H, I)}
    targets = wl["targets"].split()
    root = _Blk()
    root.model = _Blk()
    root.model.layers = nn.ModuleList()
    g = torch.Generator(device=device)
    for li in range(wl["layers"]):
        blk = _Blk()
        blk.self_attn = _Blk()
        blk.mlp = _Blk()
        for name in ("q_proj", "k_proj", "v_proj", "o_proj", "gate_proj", "up_proj", "down_proj"):
            if name not in targets:
                continue
            out, inn = shapes[name]
            lin = nn.Linear(inn, out, bias=False, device="meta")
            # an independent stream per module (hash of its full name): every projection of every
            # layer is a distinct matrix, like a loaded checkpoint's
            g.manual_seed(seed * 1000003 + zlib.crc32(f"model.layers.{li}.{name}".encode()))
            w = torch.empty(out, inn, device=device, dtype=torch.float32)
            w.normal_(0.0, 0.02, generator=g)
            lin.weight = nn.Parameter(w.to(dt), requires_grad=False)
            setattr(blk.self_attn if name in ("q_proj", "k_proj", "v_proj", "o_proj") else blk.mlp, name, lin)
        root.model.layers.append(blk)
    return root, targets


def synthetic_micro_batches(n, batch, max_len, seed):
    """Instruction-shaped lengths: prompt U[32,256] + response U[32,256], truncated
    to max_len.  The reference's collator right-pads each micro-batch to its LONGEST sample
    (torch.nn.utils.rnn.pad_sequence, hp:190-201), so a micro-batch is batch x max(len) rows of
    activations.  Returns (attention-mask token count, padded row count) per micro-batch."""
    g = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        lens = np.minimum(g.integers(32, 257, batch) + g.integers(32, 257, batch), max_len)
        out.append((int(lens.sum()), int(batch * lens.max())))
    return out


HOT_KERNELS = ("probe_sweep_a", "probe_sweep_b", "probe_sweep_c", "probe_p1", "probe_p2", "probe_finish",
               "probe_reduce",
               "delta_gemm", "delta_gemm_multiseg", "delta_pack", "adam", "merge", "fold_bf16")
# hot-path COMPONENTS (one launch set each): the probe of one group = its phase launches
COMPONENTS = {"probe": ("probe_sweep_a", "probe_reduce", "probe_sweep_b", "probe_sweep_c", "probe_finish",
                        "probe_p1", "probe_p2"),
              "delta": ("delta_gemm", "delta_gemm_multiseg", "delta_pack"), "adam": ("adam",), "merge": ("merge", "fold_bf16")}


def kernel_source_digest():
    """sha256 of the step kernels' sources (hd-pissa_amd/csrc, include): a PMC profile is used for the
    roofline's `traffic` only if it was recorded on these exact sources.  K1 (hdp_svd.hip) is left out: the
    PMC passes run `--init random`, so no counter they record comes from it."""
    import glob
    import hashlib
    h = hashlib.sha256()
    srcs = [f for f in glob.glob(os.path.join(ROOT, "hd-pissa_amd", "csrc", "*")) if os.path.basename(f) != "hdp_svd.hip"]
    for f in sorted(srcs) + [os.path.join(ROOT, "include", "hdpissa.h")]:
        h.update(os.path.basename(f).encode())
        h.update(open(f, "rb").read())
    return h.hexdigest()[:16]


PMC_ROUND = "r06"


def pmc_key(workload, exchange):
    """The PMC profile a kernel's traffic comes from: the bench command's own exchange leg
    (gather: profiles/<round>_pmc_bench_<workload>.json; allreduce -- the north-star contract's
    K4 STORE + K5 merge: ..._<workload>_allreduce.json, a pass over `bench.py --exchange allreduce`)."""
    return workload if exchange == "gather" else f"{workload}@allreduce"


def pmc_summary_path(key):
    wl, _, leg = key.partition("@")
    return os.path.join(ROOT, "profiles", f"{PMC_ROUND}_pmc_bench_{wl}{'_' + leg if leg else ''}.json")


_PMC = {}


def pmc_entry(workload, name):
    """PMC measurements of THIS bench command (tools/pmc_bench.sh -> tools/pmc_bench_summary.py):
    per kernel family the HBM bytes / algorithmic bytes (2 x FETCH_SIZE + WRITE_SIZE) and the MFMA
    busy fraction (SQ_VALU_MFMA_BUSY_CYCLES over the SIMD-cycles of the launches).  None unless the
    profile was taken on the current kernel sources (its `source_digest`)."""
    if workload not in _PMC:
        try:
            d = json.load(open(pmc_summary_path(workload)))
        except (OSError, ValueError):
            d = None
        if d is not None and d.get("source_digest") != kernel_source_digest():
            d = None
        _PMC[workload] = d
    d = _PMC[workload]
    if d is None:
        return None, None
    return d.get("traffic_over_algorithmic", {}).get(name), d.get("mfma_busy", {}).get(name)


def roofline_entry(name, bytes_, flop, seconds, launches, workload, math, pmc_names=None):
    """One roofline entry: ALGORITHMIC bytes and f32-equivalent flops per launch over the average
    launch duration; bound = whichever ceiling the arithmetic intensity reaches first (HBM at 8 TB/s
    or the MFMA ceiling of the math the kernel runs)."""
    peak_m = PEAK_MFMA_TFS[math]
    ridge = peak_m * 1e12 / (PEAK_HBM_GBS * 1e9)  # flop per byte
    traffic, src, busy = 0.0, None, {}
    for n, nb in (pmc_names or [(name, bytes_)]):
        ratio, mf = pmc_entry(workload, n)
        busy[n] = mf
        if nb == 0 and pmc_names:  # a phase with no algorithmic bytes adds none (and has no ratio)
            continue
        if ratio is None or traffic is None:
            traffic = None
            continue
        traffic += ratio * nb
        src = os.path.relpath(pmc_summary_path(workload), ROOT)
    per = dict(bytes=bytes_, flop=flop, avg_us=round(seconds * 1e6, 2), launches=launches,
               intensity_flop_per_byte=round(flop / max(bytes_, 1.0), 2), ridge_flop_per_byte=round(ridge, 2))
    extra = dict(traffic=None if traffic is None else round(traffic), traffic_source=src,
                 mfma_busy=busy.get(name) if pmc_names is None else busy, math=math, per_launch=per)
    # a kernel whose MEASURED traffic already moves >= 4.5 TB/s is bound by HBM whatever its algorithmic
    # intensity says (the bf16 r = 64 / 128 probes read X and G several times per group)
    traffic_bound = traffic is not None and traffic / seconds >= TRAFFIC_BOUND_BPS
    if traffic is not None:
        per["traffic_TBps"] = round(traffic / seconds / 1e12, 2)
    if flop / max(bytes_, 1.0) > ridge and not traffic_bound:
        ach = flop / seconds / 1e12
        return dict(kernel=name, bound="mfma", achieved=round(ach, 2), peak=round(peak_m, 1), unit="TFLOP/s",
                    frac=round(ach / peak_m, 4), hbm_GBps=round(bytes_ / seconds / 1e9, 1), **extra)
    ach = bytes_ / seconds / 1e9
    if traffic_bound and flop / max(bytes_, 1.0) > ridge:
        extra["bound_reason"] = (f"PMC traffic {traffic / seconds / 1e12:.2f} TB/s >= {TRAFFIC_BOUND_BPS / 1e12} TB/s: "
                                 f"traffic-bound (MFMA basis frac {flop / seconds / 1e12 / peak_m:.3f})")
    return dict(kernel=name, bound="hbm", achieved=round(ach, 1), peak=PEAK_HBM_GBS, unit="GB/s",
                frac=round(ach / PEAK_HBM_GBS, 4), mfma_TFs=round(flop / seconds / 1e12, 2), **extra)


def roofline_for(name, s, workload, math="f32"):
    """Roofline entry of one kernel from the library's live HIP-event timing (hdp_timing_*)."""
    return roofline_entry(name, s["bytes_per_launch"], s["flop_per_launch"], s["avg_us"] * 1e-6, s["launches"],
                          workload, math)


def probe_component(hot, probe_bytes_alg, workload, math):
    """The probe as ONE component: per group (one launch set = sweep A, reduce, B, reduce, C,
    finish), ALGORITHMIC bytes = every distinct X and every G read once; flops = the f32-equivalent
    products of the set; duration = the summed HIP-event time of the set's launches.  traffic = the
    PMC-measured HBM bytes of every launch of the set (bench-command profile)."""
    names = [n for n in COMPONENTS["probe"] if n in hot]
    first = next(n for n in ("probe_sweep_a", "probe_p1") if n in hot)
    sets = hot[first]["launches"]
    dur = sum(hot[n]["total_ms"] for n in names) * 1e-3 / sets
    flop = sum(hot[n]["flop_per_launch"] * hot[n]["launches"] for n in names) / sets
    pmc = [(n, hot[n]["bytes_per_launch"] * hot[n]["launches"] / sets) for n in names]
    e = roofline_entry("probe (K2 group: " + " + ".join(names) + ")", probe_bytes_alg / sets, flop, dur, sets,
                       workload, math, pmc_names=pmc)
    e["per_launch"]["phases_us"] = {n: round(hot[n]["total_ms"] * 1e3 / sets, 2) for n in names}
    return e


class _RandomFactorOps:
    """--init random (profiling runs only): the op set with svd_topk_batch replaced by random
    factors of the right shapes -- the hot path's traffic does not depend on their values."""

    def __init__(self, ops):
        self._ops = ops

    def __getattr__(self, k):
        return getattr(self._ops, k)

    def svd_topk_batch(self, Ws, r, nranks):
        out = []
        for W in Ws:
            o, i = W.shape
            g = torch.Generator(device=W.device)
            g.manual_seed(o * 7 + i)
            A_all = torch.randn(r * nranks, i, device=W.device, generator=g) * 0.05
            B_all = torch.randn(nranks, o, r, device=W.device, generator=g) * 0.05
            out.append((A_all, B_all, torch.ones(r * nranks, dtype=torch.float64, device=W.device)))
        return out


# ------------------------------------------------------------------------------------------
def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(wl, micro, T, tokens_per_micro, wn):
    """The reference algorithm on the host cores (oracle restatement, float32 numpy/BLAS):
    sample = one decoder layer's targeted modules: the dense adapter fwd/bwd of hp:139 for ONE
    micro-batch + Adam + the rank loop hp:389-394 at world size wn; scaled to the workload's
    step (micro-batches x layers).  Timed twice: with every BLAS thread this process has (the
    reported `value`) and with one thread.  kind = "port"."""
    from oracle import hdpissa_oracle as O
    try:
        from threadpoolctl import threadpool_info, threadpool_limits
        cores = max([i.get("num_threads", 1) for i in threadpool_info() if i.get("user_api") == "blas"] or [1])
    except Exception:  # pragma: no cover
        threadpool_limits = None
        cores = int(os.environ.get("OMP_NUM_THREADS", "1"))
    H, I, KV, r = wl["hidden"], wl["inter"], wl["kv"], wl["r"]
    shapes = {"q_proj": (H, H), "k_proj": (KV, H), "v_proj": (KV, H), "o_proj": (H, H),
              "gate_proj": (I, H), "up_proj": (I, H), "down_proj": (H, I)}

    def sample():
        g = np.random.default_rng(0)
        t_probe = t_step = 0.0
        for name in wl["targets"].split():
            out, inn = shapes[name]
            X = g.standard_normal((T, inn), dtype=np.float32)
            G = g.standard_normal((T, out), dtype=np.float32)
            A = [g.standard_normal((r, inn), dtype=np.float32) * 0.1 for _ in range(wn)]
            B = [g.standard_normal((out, r), dtype=np.float32) * 0.1 for _ in range(wn)]
            W = g.standard_normal((out, inn), dtype=np.float32) * 0.02
            t0 = time.perf_counter()
            gA, gB = O.probe_dense_adapter_only(X, G, A[0], B[0], 1.0)
            t1 = time.perf_counter()
            dA, dB = [], []
            for i in range(wn):
                _, _, da = O.adam_factors(gA, np.zeros_like(gA), np.zeros_like(gA), 1, 2e-5)
                _, _, db = O.adam_factors(gB, np.zeros_like(gB), np.zeros_like(gB), 1, 2e-5)
                dA.append(da)
                dB.append(db)
            O.merge(W, O.delta_w(dA, dB, A, B, wl["dtype"]), wl["dtype"])
            t2 = time.perf_counter()
            t_probe += t1 - t0
            t_step += t2 - t1
        layers = wl["layers"]
        step_s = micro * layers * t_probe + layers * t_step
        return t_probe, t_step, step_s, micro * tokens_per_micro / step_s

    tp, ts, step_s, value = sample()
    one = None
    if threadpool_limits is not None and cores > 1:
        with threadpool_limits(limits=1, user_api="blas"):
            tp1, ts1, step1, value1 = sample()
        one = dict(value=round(value1, 3), cores=1, sample_s=round(tp1 + ts1, 2), step_s=round(step1, 1))
    return dict(value=round(value, 2), unit="tokens/s", cores=int(cores), kind="port", cpu_model=_cpu_model(),
                one_thread=one,
                sample=(f"1 decoder layer ({len(wl['targets'].split())} modules), T={T}: reference dense adapter "
                        f"fwd/bwd (1 micro-batch) {tp:.2f}s + Adam/rank-loop dW/merge at Wn={wn} "
                        f"{ts:.2f}s; scaled x{micro} micro-batches x {wl['layers']} layers -> {step_s:.1f}s/step"))


def ref_torch_gpu(layers, Xs, Gs, rows, wn, tokens, device, probe=True, world=1):
    """The reference's own algorithm with torch ops on this GPU (the >=10x target's
    denominator): dense adapter fwd/bwd terms of hp:139 per module per micro-batch, then
    hp:352-398 (Adam as ~20 elementwise ops, 4 all_gathers, zeros_like, rank loop of 3 GEMMs,
    merge).  Runs on a scratch copy of W for one timed step.  world > 1: the all_gathers are
    real torch.distributed (RCCL) collectives, as in the reference; world == 1 with wn > 1:
    the gathered lists are local copies (rank loop of a wn-GPU run, exchange not timed)."""
    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    a0, a1, a2 = ev(), ev(), ev()
    Ws = [L.W_res.clone() for L in layers]
    grads = [(torch.zeros_like(L.A), torch.zeros_like(L.B)) for L in layers]
    states = [[torch.zeros_like(L.A), torch.zeros_like(L.A), torch.zeros_like(L.B), torch.zeros_like(L.B)]
              for L in layers]

    def one():
        a0.record()
        for Ti in (rows if probe else ()):
            for L, X, G, (gA, gB) in zip(layers, Xs, Gs, grads):
                A, B = L.A.detach(), L.B.detach()
                M = torch.mm(B, A) * 1e-16 * L.alpha
                x32 = X[:Ti].float()
                g32 = G[:Ti].float()
                _y = torch.nn.functional.linear(x32, M)
                _dx = g32 @ M
                dM = (g32.t() @ x32) * L.alpha * 1e-16
                gB += dM @ A.t()
                gA += B.t() @ dM
        a1.record()
        lr, t, b1, b2, eps = 2e-5, 1, 0.9, 0.999, 1e-8
        for L, W, (gA, gB), st in zip(layers, Ws, grads, states):
            grad_A, grad_B = gA * 1e16, gB * 1e16
            st[0] = b1 * st[0] + (1 - b1) * grad_A
            st[1] = b2 * st[1] + (1 - b2) * (grad_A ** 2)
            st[2] = b1 * st[2] + (1 - b1) * grad_B
            st[3] = b2 * st[3] + (1 - b2) * (grad_B ** 2)
            dA = lr * (st[0] / (1 - b1 ** t)) / (torch.sqrt(st[1] / (1 - b2 ** t)) + eps)
            dB = lr * (st[2] / (1 - b1 ** t)) / (torch.sqrt(st[3] / (1 - b2 ** t)) + eps)
            A, B = L.A.detach(), L.B.detach()
            if world > 1:  # hp:379-387
                dA_l, dB_l = [torch.zeros_like(dA) for _ in range(wn)], [torch.zeros_like(dB) for _ in range(wn)]
                A_l, B_l = [torch.zeros_like(A) for _ in range(wn)], [torch.zeros_like(B) for _ in range(wn)]
                dist.all_gather(dA_l, dA)
                dist.all_gather(dB_l, dB)
                dist.all_gather(A_l, A.contiguous())
                dist.all_gather(B_l, B.contiguous())
            else:
                dA_l, dB_l = [dA.clone() for _ in range(wn)], [dB.clone() for _ in range(wn)]
                A_l, B_l = [A.clone() for _ in range(wn)], [B.clone() for _ in range(wn)]
            dW = torch.zeros_like(W)
            for i in range(wn):
                dW -= (dB_l[i] @ A_l[i] + B_l[i] @ dA_l[i] - dB_l[i] @ dA_l[i])
            W += dW.to(W.dtype)
            gA.zero_()
            gB.zero_()
        a2.record()
        torch.cuda.synchronize()
        return a0.elapsed_time(a1), a1.elapsed_time(a2)

    one()  # warm-up (allocator, library handles)
    p_ms, d_ms = one()
    del Ws
    return dict(ms_per_step=round(p_ms + d_ms, 2), dw_ms_per_step=round(d_ms, 2), probe_ms_per_step=round(p_ms, 2),
                tokens_per_s=round(tokens / ((p_ms + d_ms) / 1e3), 1), wn=wn)


def dw_emulated(layers, stepper, ops, wn, device):
    """dW aggregate + merge of a wn-GPU run on one GPU, exchange excluded: this build's K3 Adam
    + the grouped K4 plan over K = 2 r wn (every rank's factors = copies of this rank's, laid
    out like the gathered arena) vs the reference's hp:352-394 rank loop over wn copies."""
    from hdpissa_amd._lib import HDP_DW_MERGE
    arena = layers[0]._arena
    F = arena.F
    fac = arena.fac.repeat(wn)
    dlt = arena.delta.repeat(wn)
    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731

    items = []
    for i, L in enumerate(arena.layers):
        oa, ob = arena.offsets[i]
        items.append((L.out_features, L.in_features, L.r, wn, dlt[oa:], dlt[ob:], F, fac[oa:], fac[ob:], F, L.W_res))
    # what HDPissaStep runs per gathered bucket: one grouped plan (here: one bucket)
    plan = ops.delta_plan(items, HDP_DW_MERGE, layers[0].W_res.dtype == torch.bfloat16)

    def ours():
        ops.adam(arena.grad, arena.m, arena.v, arena.delta, 1, 2e-5, 0.9, 0.999, 1e-8, zero_grad=True)
        plan.run()

    ours()
    torch.cuda.synchronize()
    a, b = ev(), ev()
    a.record()
    for _ in range(3):
        ours()
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / 3
    math = plan.math()
    plan.close()
    del fac, dlt
    ref = ref_torch_gpu(layers, None, None, [], wn, 0, device, probe=False)
    return dict(wn=wn, ms=round(ms, 2), ref_ms=ref["dw_ms_per_step"], speedup=round(ref["dw_ms_per_step"] / ms, 2),
                k4_math=math,
                note="K3 + K4 (K = 2 r wn) vs reference Adam + rank loop + merge; exchange excluded from both")


def plan_math(stepper):
    """The MFMA math of the step's grouped K4 plans (their roofline ceiling)."""
    for pl in stepper.plans:
        for plans in pl.plans.values():
            for p, _ in plans:
                if hasattr(p, "math"):
                    return p.math()
    return "f32"


# ------------------------------------------------------------------------------------------
class _HipPlatform:
    """The bench's device runtime: one HIP device per process, RCCL ("nccl") process group,
    HIP events, the library's live kernel timing."""
    backend = "nccl"

    def __init__(self, local):
        torch.cuda.set_device(local)
        self.device = torch.device("cuda", local)

    def sync(self):
        torch.cuda.synchronize()

    def event(self):
        return torch.cuda.Event(enable_timing=True)

    def kernel_timing(self, **kw):
        from hdpissa_amd._lib import kernel_timing
        return kernel_timing(**kw)


class _HostEvent:
    def record(self):
        self.t = time.perf_counter()

    def elapsed_time(self, other):
        return (other.t - self.t) * 1e3


class _HostPlatform:
    """CPU harness (tests/test_bench_dist.py only): CPU tensors, gloo, the op set the test injects;
    no kernel timing.  Runs the bench's multi-rank orchestration end to end without a GPU."""
    backend = "gloo"

    def __init__(self, local):
        self.device = torch.device("cpu")

    def sync(self):
        pass

    def event(self):
        return _HostEvent()

    def kernel_timing(self, **kw):
        return {}


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def self_launch(argv, nproc, launcher=None):
    """`bench.py --gpus N` (N > 1) run without a launcher: start the N ranks as a child
    `python -m torch.distributed.run --nnodes 1 --nproc-per-node N --master-addr 127.0.0.1` over
    this same script and arguments, before this process makes any GPU call (no exec from a
    process that has touched the GPU), forward the children's output, and return the child's exit
    code.  Rank 0 prints the JSON line; the parent relays stdout unchanged.  `launcher` (tests)
    replaces the torch.distributed.run argv prefix."""
    import subprocess
    # HDP_BENCH_RANK_SCRIPT (CPU harness only, tests/bench_cpu_rank.py): the per-rank entry the
    # children run instead of this file -- it injects the test op set the product never selects
    script = os.path.abspath(os.environ.get("HDP_BENCH_RANK_SCRIPT") or __file__)
    cmd = (launcher or [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node",
                        str(nproc), "--master-addr", "127.0.0.1", "--master-port", str(_free_port())])
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # RCCL over dmabuf IPC on this pool
    env["HDP_BENCH_SELF_LAUNCHED"] = "1"
    proc = subprocess.run(cmd + [script] + list(argv), env=env)
    return proc.returncode


def main(argv=None, host_ops=None, return_state=False):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="llama2-7b", choices=sorted(WORKLOADS))
    ap.add_argument("--exchange", default="gather", choices=["gather", "allreduce"])
    ap.add_argument("--micro", type=int, default=8, help="micro-batches per rank per step (run.sh: 64 // 8)")
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--seq", type=int, default=512)
    ap.add_argument("--layers", type=int, default=None, help="override the workload's decoder-layer count (experiments)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-ref-torch", action="store_true")
    ap.add_argument("--init", default="svd", choices=["svd", "random"],
                    help="svd: the K1 SVD-slice init (default); random: random factors (PMC profiling runs only: "
                         "the counters of thousands of rocSOLVER launches would dominate the profile)")
    ap.add_argument("--timing-out", default=None, help="write the per-kernel live timing of the timed steps (JSON)")
    ap.add_argument("--no-other-exchange", action="store_true",
                    help="skip timing the dW path of the other exchange strategy (N=1 leg)")
    ap.add_argument("--profile-host", action="store_true",
                    help="cProfile the host side of the timed steps (stderr; diagnosis only)")
    ap.add_argument("--distinct-x", action="store_true",
                    help="give every module its own X (r02's layout; the probe cannot share a stream)")
    ap.add_argument("--emulate-wn", type=int, default=8,
                    help="N=1 only: also time the dW path of a WN-GPU run (rank loop of WN segments) for "
                         "this build and the reference torch path (exchange excluded from both)")
    args = ap.parse_args(argv)

    if "WORLD_SIZE" not in os.environ and args.gpus > 1 and host_ops is None:
        # no launcher: start the ranks as a child before anything here touches the GPU
        if os.environ.get("HDP_BENCH_SELF_LAUNCHED"):
            raise SystemExit("bench.py: self-launched rank without WORLD_SIZE (launcher failed to set the env)")
        raise SystemExit(self_launch(sys.argv[1:] if argv is None else argv, args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch N>1 with torch.distributed.run "
                         "(or without WORLD_SIZE set, and the bench starts its ranks itself)")
    plat = _HipPlatform(local) if host_ops is None else _HostPlatform(local)
    device = plat.device
    if world > 1:
        kw = dict(device_id=device) if device.type == "cuda" else {}
        dist.init_process_group(plat.backend, rank=rank, world_size=world, **kw)

    from hdpissa_amd import HDPissaStep, flush_probes, lr_at, replace_with_custom_layer
    kernel_timing = plat.kernel_timing

    wl = dict(WORKLOADS[args.workload])
    if args.layers:
        wl["layers"] = args.layers
    dt = getattr(torch, wl["dtype"])
    X_ES = torch.empty(0, dtype=dt).element_size()
    r, alpha = wl["r"], wl["alpha"]
    T = args.batch * args.seq
    if host_ops is None:
        from hdpissa_amd.ops import default_ops
        tops = default_ops()
    else:
        tops = host_ops

    t_init = time.time()
    model, targets = build_model(wl, device)
    init_ops = tops if args.init == "svd" else _RandomFactorOps(tops)
    layers = replace_with_custom_layer(model, targets, rank, world, r, alpha, ops=init_ops)
    for L in layers:
        L._ops = tops
    if layers:
        layers[0]._arena.probe_queue.ops = tops
    plat.sync()
    t_svd = time.time() - t_init
    stepper = HDPissaStep(model, world, rank, ops=tops, exchange=args.exchange)

    # synthetic activations / output grads (resident): one X per projection group of a decoder
    # layer (q/k/v share the attention input, gate/up the MLP input), one G per module
    g = torch.Generator(device=device)
    g.manual_seed(1234 + rank)
    Xs, Gs, xbuf = [], [], {}
    for L in layers:
        prefix, proj = L.name.rsplit(".", 1)
        key = L.name if args.distinct_x else (prefix.rsplit(".", 1)[0] + (".attn_in" if proj in ("q_proj", "k_proj", "v_proj")
                                                                          else ".mlp_in" if proj in ("gate_proj", "up_proj")
                                                                          else "." + proj))
        X = xbuf.get(key)
        if X is None:
            X = xbuf[key] = torch.empty(T, L.in_features, device=device, dtype=torch.float32).normal_(generator=g).to(dt)
        G = torch.empty(T, L.out_features, device=device, dtype=torch.float32).normal_(0, 1e-3, generator=g).to(dt)
        Xs.append(X)
        Gs.append(G)
    x_elems = sum(X.shape[1] for X in xbuf.values())  # per row: every distinct X once
    toks = synthetic_micro_batches((args.warmup + args.steps) * args.micro, args.batch, args.seq, 42 + rank)
    # every micro-batch's row views, made before the timed region (autograd hands the module
    # backward its saved X and G; slicing 2 x 224 views per micro-batch is bench overhead)
    views = {}
    for _, Ti in toks:
        if Ti not in views:
            views[Ti] = [(L, X[:Ti], G[:Ti]) for L, X, G in zip(layers, Xs, Gs)]

    total_opt_steps = 1000
    warm = int(0.03 * total_opt_steps)  # run.sh: --warmup_ratio 0.03, cosine
    t_counter = [0]
    ev = plat.event
    dw_ms = []

    mb_it = [iter(toks)]

    host_s = [0.0]
    host_parts = {"push": 0.0, "flush": 0.0, "step": 0.0}

    def one_step(timed):
        h0 = time.perf_counter()
        hp = 0.0
        for _ in range(args.micro):
            _, Ti = next(mb_it[0])  # this micro-batch's padded rows (batch x longest sample)
            for L, x, gy in views[Ti]:
                L._probe_backward(x, gy)  # what autograd calls per module backward
        h1 = time.perf_counter()
        flush_probes(model)  # the last probe group is launched here, not inside the dW timing
        h2 = time.perf_counter()
        lr = lr_at(t_counter[0], 2e-5, warm, total_opt_steps, "cosine")
        t_counter[0] += 1
        e0, e1 = ev(), ev()
        e0.record()
        stepper.step(lr, t_counter[0])
        e1.record()
        if timed:
            h3 = time.perf_counter()
            dw_ms.append((e0, e1))
            host_s[0] += h3 - h0
            # pushes include the launches of the groups flushed by a repeated module (one per
            # micro-batch after the first); flush = the last group's launch
            host_parts["push"] += h1 - h0
            host_parts["flush"] += h2 - h1
            host_parts["step"] += h3 - h2

    for _ in range(args.warmup):
        one_step(False)
    plat.sync()
    if world > 1:
        dist.barrier()
    wait_us = (lambda reset=0: 0) if host_ops is not None else (
        lambda reset=0: __import__("hdpissa_amd._lib", fromlist=["lib"]).lib().hdp_probe_host_wait_us(reset))
    wait_us(1)
    prof = None
    if args.profile_host:
        import cProfile
        prof = cProfile.Profile()
        prof.enable()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        one_step(True)
    plat.sync()
    if prof is not None:
        prof.disable()
        import pstats
        pstats.Stats(prof, stream=sys.stderr).sort_stats("tottime").print_stats(25)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    timed_mb = toks[args.warmup * args.micro:]
    # The per-kernel HIP-event timing (roofline) brackets every launch with two events: on a
    # launch-bound stretch that host work would stall the GPU, so it runs in a second,
    # identical timed region (same micro-batch lengths) instead of inside the one `value` uses.
    blocked_ms = wait_us(1) / 1e3  # host time spent waiting for the GPU (staging-ring back-pressure)
    dw_value = list(dw_ms)
    host_value = host_s[0]
    parts_value = dict(host_parts)
    dw_ms.clear()
    mb_it[0] = iter(timed_mb)
    kernel_timing(enable=True, reset=True)
    ti0 = time.perf_counter()
    for _ in range(args.steps):
        one_step(True)
    plat.sync()
    instrumented_ms = 1e3 * (time.perf_counter() - ti0) / args.steps
    ks = kernel_timing(enable=False)
    dw_ms[:] = dw_value
    host_s[0] = host_value
    host_parts.update(parts_value)
    if args.timing_out and rank == 0:
        with open(args.timing_out, "w") as f:
            json.dump(ks, f)
    legs = None
    if world == 1 and not args.no_other_exchange and host_ops is None:
        # the other exchange strategy's dW path on the same arena (north-star contract: K4 store ->
        # all-reduce (identity at N = 1) -> K5 merge; or the fused gather-merge K4)
        other = "allreduce" if args.exchange == "gather" else "gather"
        st2 = HDPissaStep(model, world, rank, ops=tops, exchange=other)
        st2.step(2e-5, t_counter[0] + 1)
        plat.sync()
        kernel_timing(enable=True, reset=True)
        e0, e1 = ev(), ev()
        e0.record()
        for i in range(args.steps):
            st2.step(2e-5, t_counter[0] + 2 + i)
        e1.record()
        plat.sync()
        ks2 = kernel_timing(enable=False)
        dw_other = e0.elapsed_time(e1) / args.steps
        legs = {args.exchange: dict(dw_ms_per_step=None), other: dict(dw_ms_per_step=round(dw_other, 3))}
        for n in ("merge", "delta_gemm", "delta_gemm_multiseg", "adam"):
            if n in ks2:
                legs[other][n] = roofline_for(n, ks2[n], pmc_key(args.workload, other),
                                              plan_math(st2) if n.startswith("delta") else "f32")
        if other == "allreduce":
            # K5 alone (inside the leg it shares HBM with the next bucket's K4 on the other stream):
            # the grouped merge of the largest bucket, timed by itself
            plan = st2.plans[0]
            a_, b_ = max(plan.a_buckets, key=lambda ab: sum(plan.arena.layers[i].W_res.numel() for i in range(*ab)))
            pairs, off = [], 0
            for i in range(a_, b_):
                L = plan.arena.layers[i]
                pairs.append((L.W_res, plan.dw_bufs[0][off:off + L.W_res.numel()].view_as(L.W_res)))
                off += L.W_res.numel()
            plan.dw_bufs[0][:off].zero_()
            tops.merge_group(pairs)
            plat.sync()
            kernel_timing(enable=True, reset=True)
            for _ in range(3):
                tops.merge_group(pairs)
            plat.sync()
            km = kernel_timing(enable=False)
            if "merge" in km:
                legs[other]["k5_merge_alone"] = roofline_for("merge", km["merge"], pmc_key(args.workload, other))
                legs[other]["k5_merge_alone"]["modules"] = b_ - a_
        del st2
    el = torch.tensor([elapsed], device=device, dtype=torch.float64)
    rows_timed = [t for _, t in timed_mb]
    tok = torch.tensor([float(sum(n for n, _ in timed_mb))], device=device, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        dist.all_reduce(tok, op=dist.ReduceOp.SUM)
    elapsed, tokens = el.item(), tok.item()

    hot = {n: s for n, s in ks.items() if n in HOT_KERNELS}
    # the probe's algorithmic bytes: every distinct X and every G once per micro-batch
    probe_xg = (x_elems + sum(L.out_features for L in layers)) * X_ES * float(sum(rows_timed))
    roof = None
    if hot:  # (the CPU harness has no kernel timing)
        comp = {c: sum(hot[n]["total_ms"] for n in names if n in hot) for c, names in COMPONENTS.items()}
        dom = max(comp, key=comp.get)
        probe_math = "f32" if wl["dtype"] == "float32" else "bf16x3"
        k4_math = plan_math(stepper)
        kmath = {n: probe_math if n.startswith("probe") else k4_math if n.startswith("delta_gemm") else "f32" for n in hot}
        pk = pmc_key(args.workload, args.exchange)
        others = {n: roofline_for(n, s, pk, kmath[n]) for n, s in hot.items()}
        if dom == "probe":
            roof = probe_component(hot, probe_xg, pk, probe_math)
        else:
            k = max((n for n in COMPONENTS[dom] if n in hot), key=lambda n: hot[n]["total_ms"])
            roof = dict(others.pop(k))
        roof["dominant_component"] = dom
        roof["component_ms_per_step"] = {c: round(v / args.steps, 3) for c, v in comp.items()}
        roof["others"] = others
        if dom != "probe" and any(n in hot for n in ("probe_sweep_a", "probe_p1")):
            roof["probe"] = probe_component(hot, probe_xg, pk, probe_math)
    dw = float(np.mean([a.elapsed_time(b) for a, b in dw_ms]))

    res = {
        "metric": "train tokens/sec (node) on the HD-PiSSA hot path, " + args.workload +
                  f" r{r} (adapter probe fwd/bwd + Adam + dW aggregate + merge); dW merge+{args.exchange} ms/step",
        "value": round(tokens / elapsed, 1),
        "unit": "tokens/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 3),
        "dw_ms_per_step": round(dw, 3),
        "host_ms_per_step": round(1e3 * host_s[0] / args.steps, 3),
        "host_ms_parts": {k: round(1e3 * v / args.steps, 3) for k, v in host_parts.items()},
        # the host's own cost: wall time of the step's host code minus the time it was blocked
        # because it had run 64 probe groups (8 steps) ahead of the GPU
        "host_blocked_ms_per_step": round(blocked_ms / args.steps, 3),
        "host_busy_ms_per_step": round(1e3 * host_s[0] / args.steps - blocked_ms / args.steps, 3),
        "instrumented_ms_per_step": round(instrumented_ms, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32" if wl["dtype"] == "float32" else "bf16 W / f32 factors",
        "data": "synthetic (random-init weights of the named architecture; instruction-shaped lengths)",
        "config": {"workload": args.workload, "model": args.workload, "global_batch": args.batch * args.micro * world,
                   "seq_len": args.seq, "padding": "per micro-batch to its longest sample (hp:190-201)",
                   "rows_per_micro_mean": round(float(np.mean(rows_timed)), 1), "micro_batches_per_rank": args.micro, "r_per_gpu": r, "alpha": alpha,
                   "modules": len(layers), "exchange": args.exchange, "parallelism": f"dp{world} (HD-PiSSA slices)",
                   "x_layout": "distinct per module" if args.distinct_x else "shared per projection group (q/k/v, gate/up)"},
        "roofline": roof,
        "init_s": round(t_svd, 2),
        "init": args.init,
    }
    if legs is not None:
        legs[args.exchange]["dw_ms_per_step"] = round(dw, 3)
        res["exchange_legs"] = legs
    if not args.no_ref_torch and host_ops is None:
        try:
            ref = ref_torch_gpu(layers, Xs, Gs, rows_timed[:args.micro], world,
                                sum(n for n, _ in timed_mb[:args.micro]), device, world=world)
            ref["speedup_dw"] = round(ref["dw_ms_per_step"] / dw, 2)
            ref["speedup_step"] = round(ref["ms_per_step"] / (1e3 * elapsed / args.steps), 2)
            res["ref_torch_gpu"] = ref
        except torch.cuda.OutOfMemoryError as e:  # pragma: no cover
            res["ref_torch_gpu"] = {"error": str(e)[:200]}
        if world == 1 and args.emulate_wn > 1:
            res["dw_emulated_wn"] = dw_emulated(layers, stepper, tops, args.emulate_wn, device)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        T_mean = int(round(float(np.mean(rows_timed))))
        res["cpu_baseline"] = cpu_baseline(wl, args.micro, T_mean, tokens / args.steps / args.micro, world)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if return_state:  # (the CPU harness inspects the trained layers; it tears the group down)
        return res, layers
    if world > 1:
        dist.destroy_process_group()
    return res


if __name__ == "__main__":
    main()
