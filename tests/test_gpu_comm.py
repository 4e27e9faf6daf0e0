"""Exchange layer on one GPU.

* RcclComm (the library's own ncclComm_t, C-ABI hdp_comm_*) at world size 1: unique-id
  shipping through torch.distributed, all-gather / all-reduce / broadcast on device buffers.
* The bucketed side-stream gather orchestration of HDPissaStep at a simulated world size 2:
  a stand-in comm makes rank 1's deltas a fixed function of rank 0's (so the expected merged
  weight is computable), which exercises multi-segment K4 launches, bucket ranges, the side
  stream and its events exactly as a real 2-rank run does.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.nn as nn

from oracle import hdpissa_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture
def pg():
    if not dist.is_initialized():
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=0, world_size=1)
    yield
    dist.destroy_process_group()


def test_rccl_comm_world1(pg):
    from hdpissa_amd.comm import RcclComm
    c = RcclComm(0, 1)
    x = torch.arange(1000, dtype=torch.float32, device=DEV)
    y = torch.zeros(1000, device=DEV)
    c.allgather(x, y)
    c.allreduce_sum(x)
    b = torch.arange(10, dtype=torch.float32, device=DEV)
    c.broadcast(b, 0)
    torch.cuda.synchronize()
    assert torch.equal(y, torch.arange(1000, dtype=torch.float32, device=DEV))
    assert torch.equal(x, torch.arange(1000, dtype=torch.float32, device=DEV))
    # the rank-ordered bf16 exchange's collectives (all-to-all of float32 blocks, byte all-gather)
    a = torch.randn(4096, device=DEV)
    a2 = torch.empty_like(a)
    c.alltoall(a, a2)
    s = torch.randn(1000, device=DEV).bfloat16()
    s2 = torch.empty_like(s)
    c.allgather_any(s, s2)
    torch.cuda.synchronize()
    assert torch.equal(a2, a) and torch.equal(s2, s)
    c.close()


class TwinComm:
    """world_size 2 stand-in: rank 1's buffer = 0.5 x rank 0's (deterministic, reconstructible)."""
    world_size, rank, name = 2, 0, "twin"

    def allgather(self, send, recv):
        n = send.numel()
        recv[:n].copy_(send)
        recv[n:2 * n].copy_(send * 0.5)

    def allreduce_sum(self, buf):
        buf.mul_(1.5)

    def broadcast(self, t, root):
        pass

    # the rank-ordered bf16 exchange: rank 1's bucket = 0.5 x rank 0's, so rank 0 receives
    # (own block 0, 0.5 x own block 0) and rank 1's folded shard is fold(block 1, 0.5 x block 1)
    def alltoall(self, send, recv):
        n = send.numel() // 2
        self._sent = send.clone()
        recv[:n].copy_(send[:n])
        recv[n:].copy_(send[:n] * 0.5)

    def allgather_any(self, send, recv):
        n = send.numel()
        recv[:n].copy_(send)
        b1 = self._sent[n:2 * n]
        recv[n:2 * n].copy_(((b1.bfloat16().float()) + b1 * 0.5).bfloat16())


def _model(shapes, dt):
    m = nn.Module()
    m.layers = nn.ModuleList()
    g = torch.Generator().manual_seed(3)
    for out, inn in shapes:
        blk = nn.Module()
        blk.q_proj = nn.Linear(inn, out, bias=False)
        with torch.no_grad():
            blk.q_proj.weight.copy_(torch.randn(out, inn, generator=g) * 0.05)
        blk.q_proj = blk.q_proj.to(DEV).to(dt).requires_grad_(False)
        m.layers.append(blk)
    return m


@pytest.mark.parametrize("exchange", ["gather", "allreduce"])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_bucketed_exchange_two_ranks(exchange, dt):
    from hdpissa_amd import HDPissaStep, replace_with_custom_layer
    shapes = [(256, 192), (320, 256), (192, 384), (256, 256)]
    model = _model(shapes, dt)
    r = 8
    assert not dist.is_initialized()  # local (unsharded) SVD init of both ranks' slices
    layers = replace_with_custom_layer(model, ["q_proj"], 0, 2, r, 16.0)
    W0 = [L.W_res.float().cpu().numpy() for L in layers]
    fac = [(L._arena.fac_all[0], L._arena.fac_all[1]) for L in layers]
    g = torch.Generator(device=DEV).manual_seed(5)
    grads = []
    for L in layers:
        L.A.grad = torch.randn(L.A.shape, generator=g, device=DEV) * 1e-14
        L.B.grad = torch.randn(L.B.shape, generator=g, device=DEV) * 1e-14
        grads.append((L.A.grad.cpu().numpy(), L.B.grad.cpu().numpy()))
    # tiny buckets: several per step, so the side-stream/event ordering is exercised
    st = HDPissaStep(model, 2, 0, comm=TwinComm(), exchange=exchange, bucket_bytes=40_000)
    assert len(st.plans[0].g_buckets if exchange == "gather" else st.plans[0].a_buckets) > 1
    lr = 1e-2
    st.step(lr, 1)
    torch.cuda.synchronize()
    for j, L in enumerate(layers):
        oa, ob = L._oa, L._ob
        A = [fac[j][i][oa:oa + r * L.in_features].view(r, -1).cpu().numpy() for i in range(2)]
        B = [fac[j][i][ob:ob + L.out_features * r].view(-1, r).cpu().numpy() for i in range(2)]
        z = np.zeros_like
        _, _, dA = O.adam_factors(grads[j][0], z(grads[j][0]), z(grads[j][0]), 1, lr)
        _, _, dB = O.adam_factors(grads[j][1], z(grads[j][1]), z(grads[j][1]), 1, lr)
        if exchange == "gather":
            dtn = "bfloat16" if dt == torch.bfloat16 else "float32"
            dW = O.delta_w([dA, dA * 0.5], [dB, dB * 0.5], A, B, dtn)
            exact = O.delta_w_exact([dA, dA * 0.5], [dB, dB * 0.5], A, B)
        elif dt == torch.float32:  # this rank's dW, "all-reduced" by the stand-in (x 1.5)
            dW = 1.5 * O.delta_w([dA], [dB], A[:1], B[:1])
            exact = 1.5 * O.delta_w_exact([dA], [dB], A[:1], B[:1])
        else:  # rank-ordered bf16: fold(t0, 0.5 t0), t0 = this rank's float32 term
            t0 = O.delta_w([dA], [dB], A[:1], B[:1])
            dW = O.round_bf16(O.round_bf16(t0) + 0.5 * t0)
        got = L.W_res.float().cpu().numpy()
        if dt == torch.float32:
            assert O.rel_err(got - W0[j], exact) < 1e-4, j
        else:
            ref = O.merge(W0[j], dW, "bfloat16")
            assert O.rel_err(got, ref) < 2e-2 and np.mean(got != ref) < 0.02, j
