"""Diagnosis of the K2 team kernel (measurement tool): runs one LLaMA-2-7B probe group (224
modules, T rows) with HDP_TM_TRACE=1 and prints where the time of a step goes, from the
per-step s_memrealtime stamps (100 MHz) of streaming wave 0 and the step's publisher wave.

  python tools/team_trace.py [T] [layers]
"""
import ctypes
import os
import sys

os.environ["HDP_TM_TRACE"] = "1"
os.environ["HDP_PROBE_PATH"] = "team"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hd-pissa_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from hdpissa_amd.ops import default_ops  # noqa: E402
from hdpissa_amd._lib import lib  # noqa: E402

T = int(sys.argv[1]) if len(sys.argv) > 1 else 672
layers = int(sys.argv[2]) if len(sys.argv) > 2 else 32
dev = torch.device("cuda:0")
ops = default_ops()
shapes = ([(4096, 4096)] * 4 + [(4096, 11008)] * 2 + [(11008, 4096)]) * layers
items = []
for inn, out in shapes:
    X = torch.randn(T, inn, device=dev)
    G = torch.randn(T, out, device=dev)
    A = torch.randn(16, inn, device=dev) * 0.1
    Bt = torch.randn(16, out, device=dev) * 0.1
    items.append((X, G, A, Bt, torch.zeros(16, inn, device=dev), torch.zeros(out, 16, device=dev), 1e-16, False))
for _ in range(2):
    ops.probe_grads_group(items)
torch.cuda.synchronize()
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ev0.record()
ops.probe_grads_group(items)
ev1.record()
torch.cuda.synchronize()
print(f"group: {len(items)} modules, T={T}: {ev0.elapsed_time(ev1):.3f} ms (with tracing)")
assert os.environ.get("HDP_TM_DBG") or lib().hdp_probe_team_errors(1) == 0
nbytes = lib().hdp_probe_team_trace(None, 0)
buf = (ctypes.c_uint64 * (nbytes // 8))()
lib().hdp_probe_team_trace(buf, nbytes)
tr = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 2048, 8).astype(np.int64)
G = tr.shape[0]
P, OI, OG, PI, PS, PC, LD, OLD = range(8)
valid = tr[:, :, P] > 0
t0 = tr[:, :, :7][tr[:, :, :7] > 0].min()
us = lambda x: x / 100.0  # noqa: E731  (100 MHz)
span = tr[:, :, :7].max() - t0
print(f"kernel span (stamps) {us(span):.1f} us over {G} workgroups; steps per WG: "
      f"{valid.sum(1).min()}-{valid.sum(1).max()}")


def stat(name, d):
    d = d[np.isfinite(d)]
    if d.size == 0:
        print(f"  {name:34s} (none)")
        return
    q = np.percentile(d, [10, 50, 90, 99])
    print(f"  {name:34s} n={d.size:7d}  p10 {q[0]:7.2f}  p50 {q[1]:7.2f}  p90 {q[2]:7.2f}  p99 {q[3]:7.2f}  mean {d.mean():7.2f} us")


def diff(a, b, mask=None):
    m = (tr[:, :, a] > 0) & (tr[:, :, b] > 0)
    if mask is not None:
        m &= mask
    return us((tr[:, :, a] - tr[:, :, b])[m].astype(np.float64))


print("per step (stream wave 0 / the step's publisher), microseconds:")
per = tr[:, 1:, P] - tr[:, :-1, P]
stat("step period (PROJ to PROJ)", us(per[(tr[:, 1:, P] > 0) & (tr[:, :-1, P] > 0)].astype(np.float64)))
stat("OUTER wait for Y", diff(OG, OI))
stat("PROJ(q) -> OUTER go(q)", diff(OG, P))
stat("PROJ w0 -> publisher in (8 arrivals)", diff(PI, P))
stat("publisher: LDS sum + sc1 store drain", diff(PS, PI))
stat("publisher: counter add round trip", diff(PC, PS))
last = tr[:, :, LD] > 0
stat("last arriver: slab loads + granules", diff(LD, PC))
stat("publisher in -> granules (last only)", diff(LD, PI))
print(f"  last-arriver share of steps: {last.sum() / max(1, (tr[:, :, PC] > 0).sum()):.3f}")
# per-round view: when does each workgroup start / end its items
