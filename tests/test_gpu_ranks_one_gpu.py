"""Ranks as processes on the one GPU of the box (2, and 8 -- the north-star node): the whole multi-rank
product path on real GPU kernels (r06).

RCCL refuses two ranks on one device, so the transport here is gloo on host copies (HostComm below,
test-only); everything else is the production path of a multi-GPU run:

* replace_with_custom_layer with a communicator: the module-sharded SVD-slice init (K1 on the module's
  owner rank j % Wn, then a broadcast of its factors to the other ranks);
* per-rank gradients, then HDPissaStep.step: K3 Adam on the device, the side-stream bucketed exchange
  (gather: all-gather of the deltas; allreduce: K4 STORE + all-reduce + K5; bf16: the rank-ordered
  all-to-all / fold / all-gather), the K = 2 r Wn multi-segment K4 plans and the merges, twice.

Expected values: the reference's rank loop (hp:356-394) from the oracle's Adam and delta formulas on
the factors the init produced (both ranks' slices: every rank holds them in fac_all), with both ranks'
gradients regenerated from their seeds.  Bars: merged W 1e-5 relative and the update 1e-4 (float32);
the update within 2e-2 with < 2 % of elements differing (bf16).  All ranks must end with bitwise-
identical W (gather; bf16 all-reduce).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
SHAPES = [("q_proj", 256, 192), ("k_proj", 128, 192), ("o_proj", 192, 320), ("up_proj", 384, 256)]


class HostComm:
    """torch.distributed (gloo) on host copies of the device buffers -- TEST ONLY (two ranks share the GPU)."""
    name = "host-gloo"

    def __init__(self, rank, world_size):
        self.rank, self.world_size = rank, world_size

    def allgather(self, send, recv):
        s = send.reshape(-1).cpu()
        outs = [torch.empty_like(s) for _ in range(self.world_size)]
        dist.all_gather(outs, s)
        recv.copy_(torch.cat(outs).to(recv.device))

    def allreduce_sum(self, buf):
        h = buf.cpu()
        dist.all_reduce(h)
        buf.copy_(h.to(buf.device))

    def broadcast(self, t, root):
        h = t.cpu()
        dist.broadcast(h, src=root)
        t.copy_(h.to(t.device))

    def alltoall(self, send, recv):
        s = send.reshape(-1).cpu()
        out = torch.empty_like(s)
        dist.all_to_all_single(out, s)
        recv.copy_(out.to(recv.device))

    def allgather_any(self, send, recv):
        s = send.reshape(-1).cpu()
        if s.dtype == torch.bfloat16:  # (gloo has no 16-bit integer / bf16 gather: move the bytes)
            s8 = s.view(torch.uint8)
            outs = [torch.empty_like(s8) for _ in range(self.world_size)]
            dist.all_gather(outs, s8)
            recv.copy_(torch.cat(outs).view(torch.bfloat16).to(recv.device))
        else:
            outs = [torch.empty_like(s) for _ in range(self.world_size)]
            dist.all_gather(outs, s)
            recv.copy_(torch.cat(outs).to(recv.device))


def _grads(L, j, rank, step):
    g = torch.Generator().manual_seed(1000 * step + 10 * j + rank)
    return (torch.randn(L.A.shape, generator=g) * 1e-14, torch.randn(L.B.shape, generator=g) * 1e-14)


def _worker(rank, wn, port, dtname, exchange, errfile):
    import sys
    for p in (HERE, os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "hd-pissa_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(2 if wn <= 2 else 1)
    dist.init_process_group("gloo", rank=rank, world_size=wn)
    try:
        import torch.nn as nn
        from helpers import rel_err
        from hdpissa_amd import HDPissaStep, replace_with_custom_layer
        from oracle import hdpissa_oracle as O
        dev = torch.device("cuda:0")
        dt = getattr(torch, dtname)
        r, lr = 16, 2e-3
        model = nn.Module()
        g = torch.Generator().manual_seed(5)  # the same base weights on both ranks
        for name, out, inn in SHAPES:
            lin = nn.Linear(inn, out, bias=False)
            with torch.no_grad():
                lin.weight.copy_(torch.randn(out, inn, generator=g) * 0.05)
            setattr(model, name, lin.to(dev).to(dt).requires_grad_(False))
        comm = HostComm(rank, wn)
        layers = replace_with_custom_layer(model, [s[0] for s in SHAPES], rank, wn, r, 16.0, comm=comm)
        # the sharded init: this rank's slice is row block `rank` of every module's (A_all, B_all); the owner
        # (j % 2) decomposed it, the other rank received it -- both must hold the owner's bits
        for j, L in enumerate(layers):
            fa = L._arena.fac_all
            own = torch.cat([fa[i][L._oa:L._ob + L.out_features * r] for i in range(wn)])
            allv = [torch.empty_like(own.cpu()) for _ in range(wn)]
            dist.all_gather(allv, own.cpu())
            assert all(torch.equal(allv[0], x) for x in allv), f"module {j}: ranks hold different factor slices"
            assert torch.equal(L.A.detach(), fa[rank][L._oa:L._oa + r * L.in_features].view(r, -1))
        W0 = [L.W_res.float().cpu().numpy() for L in layers]
        st = HDPissaStep(model, wn, rank, comm=comm, exchange=exchange, bucket_bytes=40_000)
        mv = {(i, j): ([np.zeros((r, L.in_features), np.float32), np.zeros((L.out_features, r), np.float32)],
                       [np.zeros((r, L.in_features), np.float32), np.zeros((L.out_features, r), np.float32)])
              for i in range(wn) for j, L in enumerate(layers)}
        Wref = [w.astype(np.float64) if dt == torch.float32 else w for w in W0]
        for step in (1, 2):
            for j, L in enumerate(layers):
                gA, gB = _grads(L, j, rank, step)
                L.A.grad = gA.to(dev)
                L.B.grad = gB.to(dev)
            st.step(lr, step)
            torch.cuda.synchronize()
            for j, L in enumerate(layers):
                fa = L._arena.fac_all
                A = [fa[i][L._oa:L._oa + r * L.in_features].view(r, -1).cpu().numpy() for i in range(wn)]
                B = [fa[i][L._ob:L._ob + L.out_features * r].view(-1, r).cpu().numpy() for i in range(wn)]
                dA, dB = [], []
                for i in range(wn):
                    gA, gB = (x.numpy() for x in _grads(L, j, i, step))
                    (mA, mB), (vA, vB) = mv[(i, j)]
                    mA, vA, da = O.adam_factors(gA, mA, vA, step, lr)
                    mB, vB, db = O.adam_factors(gB, mB, vB, step, lr)
                    mv[(i, j)] = ([mA, mB], [vA, vB])
                    dA.append(da)
                    dB.append(db)
                got = L.W_res.float().cpu().numpy()
                if dt == torch.float32:
                    if exchange == "gather":
                        exact = O.delta_w_exact(dA, dB, A, B)
                    else:  # every rank's float32 term, summed by the all-reduce
                        exact = sum(O.delta_w_exact([dA[i]], [dB[i]], [A[i]], [B[i]]) for i in range(wn))
                    prev = Wref[j]
                    Wref[j] = prev + exact
                    assert rel_err(got, Wref[j]) < 1e-5, (step, j, rel_err(got, Wref[j]))
                    assert rel_err(got - prev, exact) < 1e-4, (step, j, rel_err(got - prev, exact))
                    Wref[j] = got.astype(np.float64)  # continue from the kernel's W (the next step's input)
                else:
                    ref = O.merge(Wref[j], O.delta_w(dA, dB, A, B, "bfloat16"), "bfloat16")
                    upd = rel_err(got - Wref[j], ref - Wref[j])
                    diff = float(np.mean(got != ref))
                    assert upd < 2e-2 and diff < 0.02, (step, j, upd, diff)
                    Wref[j] = got
        if exchange == "gather" or dt == torch.bfloat16:
            for L in layers:
                w = L.W_res.float().cpu()
                ws = [torch.zeros_like(w) for _ in range(wn)]
                dist.all_gather(ws, w)
                assert all(torch.equal(ws[0], x) for x in ws), "ranks hold different merged weights"
    except Exception as e:  # surface the assertion text to the parent
        import traceback
        with open(errfile, "a") as f:
            f.write(f"rank {rank}: {e!r}\n{traceback.format_exc()}\n")
        raise
    finally:
        dist.destroy_process_group()


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


CASES = [(2, "float32", "gather"), (2, "float32", "allreduce"), (2, "bfloat16", "gather"), (2, "bfloat16", "allreduce"),
         (8, "float32", "gather"), (8, "bfloat16", "allreduce")]


@pytest.mark.parametrize("wn,dtname,exchange", CASES)
def test_ranks_one_gpu(wn, dtname, exchange, tmp_path):
    """wn ranks (2, and 8 = the north-star node) as wn processes sharing the GPU."""
    errfile = str(tmp_path / "err.txt")
    try:
        mp.spawn(_worker, args=(wn, _port(), dtname, exchange, errfile), nprocs=wn, join=True)
    except Exception:
        msg = open(errfile).read() if os.path.exists(errfile) else ""
        pytest.fail(f"worker failed:\n{msg}")
