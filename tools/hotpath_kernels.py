"""Run the hot-path kernels at LLaMA-2-7B layer shapes (fp32, r=16, T=672): per iteration one
decoder layer's grouped probe (3 groups), its 7 fused delta-GEMM merges (Wn=1 as one grouped
plan launch, Wn=8 as one launch per module, as the step issues them),
the K5 merge of a 64 MiB slab and one Adam launch.  Used under rocprofv3 --pmc to price HBM
traffic per kernel (the bench's roofline 'traffic' field).  The library's live timing of the
warm iterations (per kernel: launches, event time, algorithmic bytes) goes to
$HOTPATH_TIMING_OUT for tools/pmc_summary.py."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hd-pissa_amd")]
import torch  # noqa: E402
import json  # noqa: E402
from hdpissa_amd._lib import HDP_DW_MERGE, kernel_timing  # noqa: E402
from hdpissa_amd.ops import default_ops  # noqa: E402

ops = default_ops()
dev = "cuda:0"
T, r = int(os.environ.get("HOTPATH_T", "672")), 16  # bench: mean padded rows per micro-batch
shapes = [(4096, 4096)] * 4 + [(11008, 4096)] * 2 + [(4096, 11008)]
iters = int(os.environ.get("ITERS", "3"))
mods = []
for out, inn in shapes:
    X = torch.randn(T, inn, device=dev)
    G = torch.randn(T, out, device=dev) * 1e-3
    A = torch.randn(r, inn, device=dev)
    Bt = torch.randn(r, out, device=dev)
    W = torch.randn(out, inn, device=dev) * 0.02
    mods.append((out, inn, X, G, A, Bt, W))
F8 = [torch.randn(8, r * (out + inn), device=dev) * 0.1 for out, inn, *_ in mods]
D8 = [torch.randn(8, r * (out + inn), device=dev) * 1e-4 for out, inn, *_ in mods]
gA = [torch.zeros(r, m[1], device=dev) for m in mods]
gB = [torch.zeros(m[0], r, device=dev) for m in mods]
big = torch.randn(16 << 20, device=dev)
dbig = torch.randn(16 << 20, device=dev) * 1e-3
n = 40_000_000
ag, am, av, ad = (torch.randn(n, device=dev) for _ in range(4))
items1 = []
for i, (out, inn, X, G, A, Bt, W) in enumerate(mods):
    Fs, Ds = F8[i].view(-1), D8[i].view(-1)
    items1.append((out, inn, r, 1, Ds, Ds[r * inn:], 0, Fs, Fs[r * inn:], 0, W))
plan1 = ops.delta_plan(items1, HDP_DW_MERGE, False)
for it in range(iters):
    if it == 1:  # the first (cold) iteration is excluded here and in tools/pmc_summary.py
        torch.cuda.synchronize()
        kernel_timing(enable=True, reset=True)
    items = [(X, G, A, Bt, gA[i], gB[i], 1e-16, True) for i, (out, inn, X, G, A, Bt, W) in enumerate(mods)]
    for grp in (items[0:3], items[3:5], items[5:7]):
        ops.probe_grads_group(grp)
    plan1.run()  # Wn = 1: the grouped persistent K4 over the layer's 7 modules (what the step runs)
    for i, (out, inn, X, G, A, Bt, W) in enumerate(mods):  # Wn = 8: one launch per module
        Fs, Ds = F8[i].view(-1), D8[i].view(-1)
        stride = r * (out + inn)
        ops.delta_gemm(out, inn, r, 8, Ds, Ds[r * inn:], stride, Fs, Fs[r * inn:], stride, W, HDP_DW_MERGE, False)
    ops.merge(big, dbig)
    ops.adam(ag, am, av, ad, 1, 2e-5, 0.9, 0.999, 1e-8, False)
torch.cuda.synchronize()
out = os.environ.get("HOTPATH_TIMING_OUT", os.path.join(ROOT, "gpurun_out", "hotpath_timing.json"))
os.makedirs(os.path.dirname(out), exist_ok=True)
json.dump(kernel_timing(enable=False), open(out, "w"), indent=1)
print("done")
