"""Debug (measurement tool): one bf16 probe case under HDP_PROBE_K32 on/off, repeated; prints rel errors."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hd-pissa_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from hdpissa_amd.ops import default_ops  # noqa: E402
from oracle import hdpissa_oracle as O  # noqa: E402

ops = default_ops()
dev = torch.device("cuda:0")
for (T, inn, out, r) in [(1024, 256, 384, 16), (6, 48, 64, 4), (100, 130, 72, 20), (1024, 896, 128, 64)]:
    g = np.random.default_rng(T + inn + r)
    X = O.round_bf16(g.standard_normal((T, inn)).astype(np.float32))
    G = O.round_bf16(g.standard_normal((T, out)).astype(np.float32))
    A = (g.standard_normal((r, inn)) * 0.2).astype(np.float32)
    B = (g.standard_normal((out, r)) * 0.2).astype(np.float32)
    rA, rB = O.probe_grads(X, G, A, B, 4.0)
    scale = float(np.float32(4.0) * np.float32(1e-16))
    for k32 in ("1", "0"):
        os.environ["HDP_PROBE_K32"] = k32
        for tr in (False, True):
            errs = []
            for rep in range(3):
                tgA = torch.zeros(r, inn, device=dev)
                tgB = torch.zeros(out, r, device=dev)
                tB = torch.from_numpy(B).to(dev)
                Bt = tB.t().contiguous() if tr else None
                ops.probe_grads(torch.from_numpy(X).to(dev).bfloat16(), torch.from_numpy(G).to(dev).bfloat16(),
                                torch.from_numpy(A).to(dev), tB, tgA, tgB, scale, False, Bt=Bt)
                torch.cuda.synchronize()
                errs.append((O.rel_err(tgA.cpu().numpy(), rA), O.rel_err(tgB.cpu().numpy(), rB)))
            print(f"T={T} in={inn} out={out} r={r} k32={k32} transposed={tr}: " +
                  " ".join(f"({a:.1e},{b:.1e})" for a, b in errs), flush=True)
