"""Sweep P1 knobs for the grouped probe at LLaMA-2-7B layer shapes (one process per knob set,
because the knobs are read once per process).  python tools/probe_sweep.py COLS U"""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hd-pissa_amd")]
import torch  # noqa: E402
from hdpissa_amd.ops import default_ops  # noqa: E402
from hdpissa_amd._lib import kernel_timing  # noqa: E402

ops = default_ops()
dev = "cuda:0"
T, r = int(os.environ.get("PROBE_T", "672")), 16
shapes = [(4096, 4096)] * 4 + [(11008, 4096)] * 2 + [(4096, 11008)]   # (out, in) of one layer
groups = [shapes[0:3], shapes[3:5], shapes[5:7]]
bufs = []
for out, inn in shapes * 4:   # 4 layers' worth of distinct buffers (beyond the 256 MB MALL)
    bufs.append((torch.randn(T, inn, device=dev), torch.randn(T, out, device=dev) * 1e-3,
                 torch.randn(r, inn, device=dev), torch.randn(r, out, device=dev),
                 torch.zeros(r, inn, device=dev), torch.zeros(out, r, device=dev)))
items = [(X, G, A, Bt, gA, gB, 1e-16, True) for (X, G, A, Bt, gA, gB) in bufs]
# groups formed like ProbeQueue: up to 16 modules / HDP_PROBE_BUDGET_MB of X + G
budget = float(os.environ.get("HDP_PROBE_BUDGET_MB", "1536")) * (1 << 20)
grp, cur, cb = [], [], 0
for it in items:
    nb = it[0].numel() * 4 + it[1].numel() * 4
    if cur and (len(cur) >= int(os.environ.get("HDP_PROBE_GROUP", "32")) or cb + nb > budget):
        grp.append(cur)
        cur, cb = [], 0
    cur.append(it)
    cb += nb
grp.append(cur)
for _ in range(3):
    for g in grp:
        ops.probe_grads_group(g)
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
kernel_timing(enable=True, reset=True)
s.record()
for _ in range(10):
    for g in grp:
        ops.probe_grads_group(g)
e.record()
torch.cuda.synchronize()
ms = s.elapsed_time(e) / 10
byts = sum(X.numel() * 4 + G.numel() * 4 for (X, G, *_) in items)
print(f"PATH={os.environ.get('HDP_PROBE_PATH', 'sweep')} BUDGET={budget / 2**20:.0f}MB COLS={os.environ.get('HDP_P1_COLS')} "
      f"U={os.environ.get('HDP_P1_U')}: {ms:.3f} ms per 4 layers ({len(grp)} groups) -> {byts / ms / 1e6:.0f} GB/s "
      f"(X+G once)")
tot = 0.0
for k, v in kernel_timing(enable=False).items():
    tot += v["total_ms"]
    print(f"   {k:16s} {v['launches']:5d} launches  avg {v['avg_us']:8.2f} us  "
          f"{v['bytes_per_launch'] / v['avg_us'] / 1e3:8.1f} GB/s alg  {v['flop_per_launch'] / v['avg_us'] / 1e6:7.1f} TF/s")
print(f"   sum of kernel times per 4 layers: {tot / 10:.3f} ms")
