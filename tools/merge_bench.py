"""K5 merge bandwidth through the library (measurement tool): hdp_merge_group on a ~1 GiB float32 dW bucket over
bf16 or float32 W (algorithmic bytes: W read + W written + dW read), HIP events around each run.
  python tools/merge_bench.py [--dtype bf16|f32] [--reps 10]   (HDPISSA_LIB=<variant build> for A/B)"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hd-pissa_amd")]
import torch  # noqa: E402

from hdpissa_amd.ops import default_ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--bf16-dw", action="store_true", help="bf16 dW (the rank-ordered bf16 exchange's merge)")
    args = ap.parse_args()
    ops = default_ops()
    dt = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    shapes = [(4096, 4096)] * 4 + [(11008, 4096)] * 2 + [(4096, 11008)]  # one LLaMA-2-7B layer, x4 layers
    pairs = []
    for _ in range(4):
        for o, i in shapes:
            dw = torch.full((o, i), 1e-3, device="cuda")
            pairs.append((torch.zeros(o, i, device="cuda", dtype=dt), dw.bfloat16() if args.bf16_dw else dw))
    n = sum(W.numel() for W, _ in pairs)
    ops.merge_group(pairs)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(args.reps):
        ops.merge_group(pairs)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / args.reps
    byts = n * (2 * (2 if dt == torch.bfloat16 else 4) + (2 if args.bf16_dw else 4))
    print(json.dumps(dict(dtype=args.dtype, bf16_dw=args.bf16_dw, lib=os.environ.get("HDPISSA_LIB", "default"), elements=n, ms=round(ms, 3),
                          TBps=round(byts / ms / 1e9, 3), frac=round(byts / ms / 1e9 / 8.0, 3))), flush=True)


if __name__ == "__main__":
    main()
