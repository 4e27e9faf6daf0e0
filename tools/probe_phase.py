"""K2 phase timing at a BASELINE workload's module shapes, laid out like bench.py (one X per projection
group: q/k/v share the attention input, gate/up the MLP input; one G per module; the whole set is ONE
group), through the ctypes path (so HDPISSA_LIB=<ablation build> takes effect).  Measurement tool.
  python tools/probe_phase.py [--workload llama2-7b] [--layers 8] [--T 692] [--reps 10]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hd-pissa_amd")]
import torch  # noqa: E402

from bench import WORKLOADS  # noqa: E402
from hdpissa_amd._lib import kernel_timing  # noqa: E402
from hdpissa_amd.ops import default_ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="llama2-7b")
    ap.add_argument("--layers", type=int, default=8)
    ap.add_argument("--T", type=int, default=692)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--no-handoff-wait", action="store_true",
                    help="ablation: HDP_PROBE_SPIN=-1 (every hand-off wait gives up at once; results WRONG, timing only)")
    args = ap.parse_args()
    if args.no_handoff_wait:
        os.environ["HDP_PROBE_SPIN"] = "-1"
    from hdpissa_amd._lib import lib
    wl = WORKLOADS[args.workload]
    H, I, KV, r = wl["hidden"], wl["inter"], wl["kv"], wl["r"]
    dt = getattr(torch, wl["dtype"])
    ops = default_ops()
    dev = "cuda:0"
    T = args.T
    shapes = {"q_proj": (H, H), "k_proj": (KV, H), "v_proj": (KV, H), "o_proj": (H, H),
              "gate_proj": (I, H), "up_proj": (I, H), "down_proj": (H, I)}
    items, xbytes = [], 0
    for _ in range(args.layers):
        xs = {}
        for name, (out, inn) in shapes.items():
            key = "attn" if name in ("q_proj", "k_proj", "v_proj") else "mlp" if name in ("gate_proj", "up_proj") else name
            if key not in xs:
                xs[key] = torch.randn(T, inn, device=dev).to(dt)
                xbytes += xs[key].numel() * xs[key].element_size()
            G = (torch.randn(T, out, device=dev) * 1e-3).to(dt)
            xbytes += G.numel() * G.element_size()
            A = torch.randn(r, inn, device=dev) * 0.05
            Bt = torch.randn(r, out, device=dev) * 0.05
            items.append((xs[key], G, A, Bt, torch.zeros(r, inn, device=dev), torch.zeros(out, r, device=dev), 1e-16,
                          True))
    def clear():
        if args.no_handoff_wait:
            torch.cuda.synchronize()
            lib().hdp_probe_errors(1)

    for _ in range(2):
        ops.probe_grads_group(items)
        clear()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    kernel_timing(enable=True, reset=True)
    s.record()
    for _ in range(args.reps):
        ops.probe_grads_group(items)
        clear()
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / args.reps
    kt = kernel_timing(enable=False)
    phases = {k: round(v["total_ms"] * 1e3 / args.reps, 1) for k, v in kt.items()}
    print(json.dumps(dict(workload=args.workload, no_handoff_wait=args.no_handoff_wait, layers=args.layers, T=T, lib=os.environ.get("HDPISSA_LIB", "default"),
                          ms_per_group=round(ms, 3), xg_once_GBps=round(xbytes / ms / 1e6, 1),
                          phases_us_per_group=phases)), flush=True)


if __name__ == "__main__":
    main()
