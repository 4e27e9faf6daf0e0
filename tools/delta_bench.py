"""K4 microbenchmark (measurement tool, not part of the library): the grouped persistent
delta-GEMM plan vs one launch per module, at LLaMA-2-7B module shapes, float32 W.

  python tools/delta_bench.py [--layers 8] [--wn 1 8] [--pol 0 1 2 3] [--reps 5]

Prints one JSON line per configuration: ms per plan run, algorithmic GB/s (W read + write +
factors) and TFLOP/s.  HDP_DELTA_POL selects the cache policy of the float32 merge variant
(bit 0: non-temporal W stores, bit 1: non-temporal W loads).
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hd-pissa_amd")]

import torch  # noqa: E402

SHAPES = {"llama2-7b": [(4096, 4096)] * 4 + [(11008, 4096)] * 2 + [(4096, 11008)],
          "mistral-7b": [(4096, 4096), (1024, 4096), (1024, 4096), (4096, 4096)] + [(14336, 4096)] * 2 + [(4096, 14336)],
          "llama2-13b": [(5120, 5120)] * 4 + [(13824, 5120)] * 2 + [(5120, 13824)]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=8)
    ap.add_argument("--wn", type=int, nargs="+", default=[1, 8])
    ap.add_argument("--pol", type=int, nargs="+", default=[0])
    ap.add_argument("--r", type=int, default=16)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--single", action="store_true", help="also time one launch per module")
    ap.add_argument("--math", nargs="+", default=["auto"], choices=["auto", "f32", "x3", "h2"])
    ap.add_argument("--shapes", default="llama2-7b", choices=sorted(SHAPES))
    ap.add_argument("--dtype", default="f32", choices=["f32", "bf16"], help="W dtype")
    ap.add_argument("--mode", default="merge", choices=["merge", "store"])
    ap.add_argument("--round", action="store_true", help="bf16 per-rank rounding (ROUND plans, Wn > 1)")
    args = ap.parse_args()
    from hdpissa_amd._lib import HDP_DW_MERGE, HDP_DW_STORE, lib
    from hdpissa_amd.ops import default_ops
    ops = default_ops()
    dev = torch.device("cuda:0")
    r = args.r
    shapes = SHAPES[args.shapes] * args.layers
    wdt = torch.float32 if args.dtype == "f32" else torch.bfloat16
    Ws = [(torch.randn(o, i, device=dev) * 0.02).to(wdt) for o, i in shapes]
    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    for wn in args.wn:
        # arena-like layout: per module [A (r x in) | B (out x r)] for every rank segment
        sizes = [r * i + o * r for o, i in shapes]
        F = sum(sizes)
        fac = torch.randn(wn * F, device=dev) * 0.1
        dlt = torch.randn(wn * F, device=dev) * 1e-4
        items, off = [], 0
        for (o, i), W, n in zip(shapes, Ws, sizes):
            items.append((o, i, r, wn, dlt[off:], dlt[off + r * i:], F, fac[off:], fac[off + r * i:], F, W))
            off += n
        nbytes = sum(2.0 * Ws[0].element_size() * o * i + 8.0 * r * (o + i) * wn for o, i in shapes)
        flops = sum(4.0 * o * i * r * wn for o, i in shapes)
        for math, pol in [(m, p) for m in args.math for p in args.pol]:
            lib().hdp_delta_set_math({"auto": 0, "f32": 1, "x3": 2, "h2": 3}[math])
            os.environ["HDP_DELTA_POL"] = str(pol)
            plan = ops.delta_plan(items, HDP_DW_MERGE if args.mode == "merge" else HDP_DW_STORE, args.round)
            tiles, grid = plan.tiles()
            plan.run()
            torch.cuda.synchronize()
            a, b = ev(), ev()
            a.record()
            for _ in range(args.reps):
                plan.run()
            b.record()
            torch.cuda.synchronize()
            ms = a.elapsed_time(b) / args.reps
            print(json.dumps(dict(kind="plan", shapes=args.shapes, dtype=args.dtype, r=r, mode=args.mode, wn=wn, math=math, pol=pol,
                                  round=args.round, plan_math=plan.math(), modules=len(shapes), tiles=tiles, grid=grid,
                                  ms=round(ms, 3), GBps=round(nbytes / ms / 1e6, 1), TFs=round(flops / ms / 1e9, 2))),
                  flush=True)
            plan.close()
        for math in (args.math if args.single else []):
            lib().hdp_delta_set_math({"auto": 0, "f32": 1, "x3": 2, "h2": 3}[math])

            def run_single():
                for it in items:
                    ops.delta_gemm(*it, HDP_DW_MERGE, False)
            run_single()
            torch.cuda.synchronize()
            a, b = ev(), ev()
            a.record()
            for _ in range(args.reps):
                run_single()
            b.record()
            torch.cuda.synchronize()
            ms = a.elapsed_time(b) / args.reps
            print(json.dumps(dict(kind="single", wn=wn, math=math, modules=len(shapes), ms=round(ms, 3),
                                  GBps=round(nbytes / ms / 1e6, 1), TFs=round(flops / ms / 1e9, 2))), flush=True)
        del fac, dlt


if __name__ == "__main__":
    main()
