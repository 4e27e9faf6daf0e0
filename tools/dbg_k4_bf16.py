"""Diagnostic (measurement tool): repeat the bf16 deferred-merge plan of
test_delta_plan_h2_bf16_deferred_merge several times per HDP_K4_DEFER setting and report where runs
differ (module, row, column pattern) -- run-to-run and def 0 vs def 3."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hd-pissa_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from test_gpu_kernels import _delta_operands  # noqa: E402
from hdpissa_amd._lib import HDP_DW_MERGE, HDP_MATH_H2, lib  # noqa: E402
from hdpissa_amd.ops import default_ops  # noqa: E402

shapes = [(4096, 4096, 64, 1), (520, 200, 64, 1), (1024, 1536, 72, 1), (300, 260, 128, 1), (2048, 4096, 64, 1)]
ops = default_ops()


def run(defer):
    os.environ["HDP_K4_DEFER"] = defer
    g = np.random.default_rng(31)
    items = []
    for (out, inn, r, nseg) in shapes:
        (A, B, dA, dB), oa = _delta_operands(g, out, inn, r, nseg, 3e-2)
        W = (g.standard_normal((out, inn)) * 0.05).astype(np.float32)
        items.append((out, inn, *oa, torch.from_numpy(W).cuda().bfloat16()))
    prev = lib().hdp_delta_set_math(HDP_MATH_H2)
    plan = ops.delta_plan(items, HDP_DW_MERGE, True)
    plan.run()
    torch.cuda.synchronize()
    plan.close()
    lib().hdp_delta_set_math(prev)
    return [it[-1].float().cpu().numpy() for it in items]


def diff(a, b, tag):
    for m, (x, y) in enumerate(zip(a, b)):
        bad = np.argwhere(x != y)
        if len(bad):
            rows, cols = bad[:, 0], bad[:, 1]
            print(f"  {tag} module {m} {shapes[m][:2]}: {len(bad)} differ; rows {rows.min()}..{rows.max()} "
                  f"cols {cols.min()}..{cols.max()}; row%32 {sorted(set((rows % 32).tolist()))[:12]} "
                  f"col%64 {sorted(set((cols % 64).tolist()))[:16]} first {bad[:3].tolist()}", flush=True)


base = {d: run(d) for d in ("0", "3")}
diff(base["0"], base["3"], "def0 vs def3")
for k in range(6):
    for d in ("0", "3"):
        diff(base[d], run(d), f"rep{k} def{d}")
print("done", flush=True)
