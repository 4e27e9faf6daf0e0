"""K1 truncated-path probe (r05): block Krylov vs the full batched eigensolve at the bf16 configs' k = 64 / 128.

For each (out, in, k): Gaussian W (the bench's init, std 0.02), three matrices through svd_topk_batch with the
default path (HDP_EIG_TRACE prints accept / fallback and the residual) and with HDP_EIG=full; prints both times
and the largest relative difference of the singular values and of the triplet residuals ||W v - s u|| / s.
usage: python tools/svd_kry_probe.py [--shapes 4096x4096,14336x4096] [--k 64 128] [--m M]"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "hd-pissa_amd"))


def run(ops, Ws, k):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = ops.svd_topk_batch(Ws, k, 1)
    torch.cuda.synchronize()
    return time.perf_counter() - t0, res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="4096x4096,14336x4096,5120x5120,13824x5120")
    ap.add_argument("--k", type=int, nargs="+", default=[64, 128])
    ap.add_argument("--count", type=int, default=3)
    args = ap.parse_args()
    from hdpissa_amd.ops import default_ops
    ops = default_ops()
    dev = torch.device("cuda:0")
    for sh in args.shapes.split(","):
        out, inn = map(int, sh.split("x"))
        g = torch.Generator(device=dev).manual_seed(out + inn)
        Ws = [torch.empty(out, inn, device=dev).normal_(0, 0.02, generator=g) for _ in range(args.count)]
        for k in args.k:
            os.environ["HDP_EIG"] = "full"
            run(ops, Ws[:1], k)  # warm the solver handles
            tf, rf = run(ops, Ws, k)
            os.environ.pop("HDP_EIG")
            os.environ["HDP_EIG_TRACE"] = "1"
            tk, rk = run(ops, Ws, k)
            os.environ.pop("HDP_EIG_TRACE")
            ds, rv = 0.0, 0.0
            for W, (A, B, S), (_, _, Sf) in zip(Ws, rk, rf):
                S64, Sf64 = S.double(), Sf.double()
                ds = max(ds, float(((S64 - Sf64).abs() / Sf64).max()))
                sq = S64.sqrt()
                V = (A.double() / sq[:, None]).t()
                U = B[0].double() / sq[None, :]
                res = torch.linalg.norm(W.double() @ V - U * S64[None, :], dim=0) / S64
                rv = max(rv, float(res.max()))
            print(json.dumps({"out": out, "in": inn, "k": k, "count": args.count, "full_s": round(tf, 3),
                              "krylov_s": round(tk, 3), "max_rel_dS_vs_full": ds, "max_triplet_residual": rv}),
                  flush=True)


if __name__ == "__main__":
    main()
