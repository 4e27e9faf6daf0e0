"""Sweep P1 knobs for the grouped probe at LLaMA-2-7B layer shapes (one process per knob set,
because the knobs are read once per process).  python tools/probe_sweep.py COLS U"""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hd-pissa_amd")]
import torch  # noqa: E402
from hdpissa_amd.ops import default_ops  # noqa: E402

ops = default_ops()
dev = "cuda:0"
T, r = 1024, 16
shapes = [(4096, 4096)] * 4 + [(11008, 4096)] * 2 + [(4096, 11008)]   # (out, in) of one layer
groups = [shapes[0:3], shapes[3:5], shapes[5:7]]
bufs = []
for out, inn in shapes * 4:   # 4 layers' worth of distinct buffers (beyond the 256 MB MALL)
    bufs.append((torch.randn(T, inn, device=dev), torch.randn(T, out, device=dev) * 1e-3,
                 torch.randn(r, inn, device=dev), torch.randn(r, out, device=dev),
                 torch.zeros(r, inn, device=dev), torch.zeros(out, r, device=dev)))
items = [(X, G, A, Bt, gA, gB, 1e-16, True) for (X, G, A, Bt, gA, gB) in bufs]
grp = []
i = 0
for layer in range(4):
    for gsz in (3, 2, 2):
        grp.append(items[i:i + gsz])
        i += gsz
for _ in range(3):
    for g in grp:
        ops.probe_grads_group(g)
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(10):
    for g in grp:
        ops.probe_grads_group(g)
e.record()
torch.cuda.synchronize()
ms = s.elapsed_time(e) / 10
byts = sum(X.numel() * 4 + G.numel() * 4 for (X, G, *_) in items)
print(f"COLS={os.environ.get('HDP_P1_COLS')} U={os.environ.get('HDP_P1_U')}: {ms:.3f} ms per 4 layers "
      f"({len(grp)} groups) -> {byts / ms / 1e6:.0f} GB/s (X+G once)")
