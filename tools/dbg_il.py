"""Debug helper (measurement tool): bf16 single-segment H2 merges with the immediate (DEF 0) and deferred (DEF 3)
epilogues against the oracle, per module: error vs the reference and where the two differ (row / column mod the
256 x 128 workgroup tile)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hd-pissa_amd"), os.path.join(ROOT, "tests")]
from oracle import hdpissa_oracle as O  # noqa: E402
from test_gpu_kernels import _delta_operands, _t  # noqa: E402
from hdpissa_amd._lib import HDP_DW_MERGE, HDP_MATH_H2, lib  # noqa: E402
from hdpissa_amd.ops import default_ops  # noqa: E402

ops = default_ops()
shapes = [(4096, 4096, 64, 1), (520, 200, 64, 1), (1024, 1536, 72, 1), (300, 260, 128, 1), (2048, 4096, 64, 1)]
runs = {}
for defer in ("0", "3", "3r"):
    os.environ["HDP_K4_DEFER"] = defer[0]
    g = np.random.default_rng(31)
    items, refs = [], []
    for (out, inn, r, nseg) in shapes:
        (A, B, dA, dB), ops_args = _delta_operands(g, out, inn, r, nseg, 3e-2)
        W = (g.standard_normal((out, inn)) * 0.05).astype(np.float32)
        items.append((out, inn, *ops_args, _t(W).bfloat16()))
        refs.append((W, A, B, dA, dB))
    lib().hdp_delta_set_math(HDP_MATH_H2)
    plan = ops.delta_plan(items, HDP_DW_MERGE, True)
    plan.run()
    torch.cuda.synchronize()
    plan.close()
    runs[defer] = [it[-1].float().cpu().numpy() for it in items]
for m, (W, A, B, dA, dB) in enumerate(refs):
    Wb = _t(W).bfloat16().float().cpu().numpy()
    ref = O.merge(Wb, O.delta_w(dA, dB, A, B, "bfloat16"), "bfloat16")
    line = [f"m{m} {W.shape}"]
    for k in runs:
        got = runs[k][m]
        line.append(f"D{k}: rel {O.rel_err(got - Wb, ref - Wb):.2e} diff {np.mean(got != ref):.4f}")
    d = runs["0"][m] != runs["3"][m]
    if d.any():
        rr, cc = np.nonzero(d)
        line.append(f"0!=3 at {d.sum()} elems rows%256 {np.unique(rr % 256)[:12]} cols%128 {np.unique(cc % 128)[:12]} "
                    f"row-tiles {np.unique(rr // 256)[:8]} col-tiles {np.unique(cc // 128)[:8]}")
    print(" | ".join(line), flush=True)
