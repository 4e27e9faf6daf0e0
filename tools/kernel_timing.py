"""Per-kernel timing at LLaMA-2-7B module shapes (dev tool; HIP events on the launch stream).

python tools/kernel_timing.py [--quick]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hd-pissa_amd")]

import torch  # noqa: E402

from hdpissa_amd._lib import HDP_DW_MERGE, HDP_DW_STORE  # noqa: E402
from hdpissa_amd.ops import default_ops  # noqa: E402


def timeit(fn, iters=10, warm=2):
    for _ in range(warm):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    args = ap.parse_args()
    ops = default_ops()
    dev = "cuda:0"
    res = {}
    # merge
    for dt in (torch.float32, torch.bfloat16):
        n = 11008 * 4096
        W = torch.randn(n, device=dev).to(dt)
        dW = torch.randn(n, device=dev) * 1e-3
        ms = timeit(lambda: ops.merge(W, dW), 20)
        bpe = 12 if dt == torch.float32 else 8
        res[f"merge_{dt}"] = dict(ms=ms, GBs=n * bpe / ms / 1e6)
    # delta gemm
    for (out, inn) in ((4096, 4096), (11008, 4096), (4096, 11008)):
        for nseg in (1, 2, 4, 8):
            r = 16
            F = r * inn + out * r
            fac = torch.randn(nseg, F, device=dev) * 0.1
            dl = torch.randn(nseg, F, device=dev) * 1e-4
            W = torch.randn(out, inn, device=dev) * 0.02
            fd, ff = dl.view(-1), fac.view(-1)
            f = lambda: ops.delta_gemm(out, inn, r, nseg, fd, fd[r * inn:], F, ff, ff[r * inn:], F, W, HDP_DW_MERGE, False)
            ms = timeit(f, 10)
            flops = 4.0 * out * inn * r * nseg
            res[f"delta_merge_{out}x{inn}_w{nseg}"] = dict(ms=ms, TFs=flops / ms / 1e9, GBs=8 * out * inn / ms / 1e6)
            if nseg == 1:
                D = torch.empty(out, inn, device=dev)
                f2 = lambda: ops.delta_gemm(out, inn, r, 1, fd, fd[r * inn:], F, ff, ff[r * inn:], F, D, HDP_DW_STORE, False)
                ms2 = timeit(f2, 10)
                res[f"delta_store_{out}x{inn}"] = dict(ms=ms2, GBs=4 * out * inn / ms2 / 1e6)
    # probe
    for (out, inn) in ((4096, 4096), (11008, 4096)):
        for r in (16, 64, 128):
            T = 1024
            X = torch.randn(T, inn, device=dev)
            G = torch.randn(T, out, device=dev)
            A = torch.randn(r, inn, device=dev)
            B = torch.randn(out, r, device=dev)
            gA = torch.zeros_like(A)
            gB = torch.zeros_like(B)
            ms = timeit(lambda: ops.probe_grads(X, G, A, B, gA, gB, 1e-16, True), 10)
            res[f"probe_T{T}_{out}x{inn}_r{r}"] = dict(ms=ms, TFs=4.0 * T * r * (inn + out) / ms / 1e9,
                                                        GBs=2 * 4 * T * (inn + out) / ms / 1e6)
    # adam
    n = 40_000_000
    g = torch.randn(n, device=dev)
    m = torch.zeros(n, device=dev)
    v = torch.zeros(n, device=dev)
    d = torch.zeros(n, device=dev)
    ms = timeit(lambda: ops.adam(g, m, v, d, 1, 2e-5, 0.9, 0.999, 1e-8, False), 10)
    res["adam_40M"] = dict(ms=ms, GBs=24 * n / ms / 1e6)
    # svd
    for (out, inn, k) in ((4096, 4096, 16), (4096, 4096, 128), (11008, 4096, 16), (4096, 11008, 128)):
        if args.quick and k > 16:
            continue
        W = torch.randn(out, inn, device=dev) * 0.02
        ops.svd_topk(W, k, 1)
        torch.cuda.synchronize()
        t0 = time.time()
        ops.svd_topk(W, k, 1)
        torch.cuda.synchronize()
        res[f"svd_{out}x{inn}_k{k}"] = dict(ms=(time.time() - t0) * 1e3)
    for k, v in res.items():
        print(k, json.dumps({a: round(b, 4) for a, b in v.items()}))


if __name__ == "__main__":
    main()
