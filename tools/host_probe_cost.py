"""Host cost of one module backward on the probe path (measurement tool): times N calls of
CustomLinearLayer._probe_backward on resident X / G and prints a cProfile summary."""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hd-pissa_amd")]
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

from hdpissa_amd import flush_probes, replace_with_custom_layer  # noqa: E402

dev = torch.device("cuda:0")
root = nn.Module()
for i in range(16):
    lin = nn.Linear(512, 512, bias=False).to(dev)
    lin.weight.requires_grad = False
    setattr(root, f"m{i}_proj", lin)
layers = replace_with_custom_layer(root, ["_proj"], 0, 1, 16, 16.0)
X = torch.randn(64, 512, device=dev)
G = torch.randn(64, 512, device=dev)
for L in layers:
    L._probe_backward(X, G)
flush_probes(root)
torch.cuda.synchronize()
N = 4000
t0 = time.perf_counter()
for k in range(N // 16):
    for L in layers:
        L._probe_backward(X, G)
t1 = time.perf_counter()
flush_probes(root)
torch.cuda.synchronize()
print(f"host us per module backward: {1e6 * (t1 - t0) / N:.2f}")
pr = cProfile.Profile()
pr.enable()
for k in range(N // 16):
    for L in layers:
        L._probe_backward(X, G)
pr.disable()
flush_probes(root)
torch.cuda.synchronize()
pstats.Stats(pr).sort_stats("tottime").print_stats(14)
