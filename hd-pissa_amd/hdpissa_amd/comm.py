"""Cross-rank exchange for the HD-PiSSA step (replaces hp:379-387).

``RcclComm``   -- the library's own RCCL communicator (C-ABI ``hdp_comm_*``): collectives
                  enqueued on torch's current HIP stream (a dedicated side stream in the step),
                  so they overlap the delta GEMMs running on the compute stream.  The
                  ncclUniqueId is created on rank 0 and shipped over the already-initialised
                  torch.distributed default group (the reference's env:// rendezvous).
``TorchComm``  -- the same collectives through torch.distributed (any backend; gloo on
                  CPU for the multi-process host tests, RCCL on GPU when HDP_COMM=torch).
``LocalComm``  -- world_size == 1: every collective is the identity.
"""
from __future__ import annotations

import ctypes
import os
import sys

import torch
import torch.distributed as dist


class LocalComm:
    world_size = 1
    rank = 0
    name = "local"

    def allgather(self, send: torch.Tensor, recv: torch.Tensor) -> None:
        if recv.data_ptr() != send.data_ptr():
            recv.copy_(send.reshape(-1))

    def allreduce_sum(self, buf: torch.Tensor) -> None:
        return None

    def broadcast(self, t: torch.Tensor, root: int) -> None:
        return None

    def alltoall(self, send: torch.Tensor, recv: torch.Tensor) -> None:
        if recv.data_ptr() != send.data_ptr():
            recv.copy_(send)

    def allgather_any(self, send: torch.Tensor, recv: torch.Tensor) -> None:
        self.allgather(send, recv)


class TorchComm:
    name = "torch"

    def __init__(self, rank: int, world_size: int, group=None):
        self.rank, self.world_size, self.group = rank, world_size, group

    def allgather(self, send: torch.Tensor, recv: torch.Tensor) -> None:
        n = send.numel()
        outs = list(recv.view(self.world_size, n).unbind(0))
        dist.all_gather(outs, send.reshape(-1), group=self.group)

    def allreduce_sum(self, buf: torch.Tensor) -> None:
        dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.group)

    def broadcast(self, t: torch.Tensor, root: int) -> None:
        dist.broadcast(t, src=root, group=self.group)

    def alltoall(self, send: torch.Tensor, recv: torch.Tensor) -> None:
        """Equal blocks: send block j -> rank j, recv block i <- rank i (flat tensors)."""
        dist.all_to_all_single(recv, send, group=self.group)

    def allgather_any(self, send: torch.Tensor, recv: torch.Tensor) -> None:
        """allgather of any dtype (the folded bf16 shards)."""
        dist.all_gather_into_tensor(recv, send.reshape(-1), group=self.group)


class RcclComm:
    name = "rccl"

    def __init__(self, rank: int, world_size: int, group=None):
        from ._lib import check, lib
        self.rank, self.world_size = rank, world_size
        L = lib()
        uid = (ctypes.c_ubyte * 128)()
        obj = [b""]
        if rank == 0:  # a failure here is broadcast too (an empty id), so no rank waits on a broadcast that never comes
            obj = [bytes(uid) if L.hdp_comm_unique_id(uid, 128) == 0 else b""]
        dist.broadcast_object_list(obj, src=0, group=group)
        if len(obj[0]) != 128:
            raise RuntimeError("hdp_comm_unique_id failed on rank 0")
        uid = (ctypes.c_ubyte * 128).from_buffer_copy(obj[0])
        h = ctypes.c_void_p()
        check(L.hdp_comm_init(ctypes.byref(h), uid, 128, world_size, rank), "hdp_comm_init")
        self._h = h
        self._check, self._lib = check, L

    @staticmethod
    def _stream() -> int:
        return torch.cuda.current_stream().cuda_stream

    def allgather(self, send: torch.Tensor, recv: torch.Tensor) -> None:
        assert send.dtype == torch.float32 and recv.numel() == send.numel() * self.world_size
        self._check(self._lib.hdp_allgather_f32(self._h, send.data_ptr(), recv.data_ptr(), send.numel(),
                                                self._stream()), "hdp_allgather_f32")

    def allreduce_sum(self, buf: torch.Tensor) -> None:
        assert buf.dtype == torch.float32
        self._check(self._lib.hdp_allreduce_sum_f32(self._h, buf.data_ptr(), buf.numel(), self._stream()),
                    "hdp_allreduce_sum_f32")

    def broadcast(self, t: torch.Tensor, root: int) -> None:
        self._check(self._lib.hdp_broadcast_bytes(self._h, t.data_ptr(), t.numel() * t.element_size(), root,
                                                  self._stream()), "hdp_broadcast_bytes")

    def alltoall(self, send: torch.Tensor, recv: torch.Tensor) -> None:
        assert send.dtype == torch.float32 and recv.dtype == torch.float32
        assert send.numel() == recv.numel() and send.numel() % self.world_size == 0
        self._check(self._lib.hdp_alltoall_f32(self._h, send.data_ptr(), recv.data_ptr(),
                                               send.numel() // self.world_size, self._stream()), "hdp_alltoall_f32")

    def allgather_any(self, send: torch.Tensor, recv: torch.Tensor) -> None:
        nb = send.numel() * send.element_size()
        assert recv.numel() * recv.element_size() == nb * self.world_size
        self._check(self._lib.hdp_allgather_bytes(self._h, send.data_ptr(), recv.data_ptr(), nb, self._stream()),
                    "hdp_allgather_bytes")

    def close(self) -> None:
        if getattr(self, "_h", None) is not None:
            self._lib.hdp_comm_destroy(self._h)
            self._h = None


def make_comm(rank: int, world_size: int, device: torch.device, group=None):
    """Default communicator: identity at world_size 1; the library's RCCL communicator on
    a HIP device (HDP_COMM=torch selects torch.distributed instead); torch.distributed
    for CPU tensors (the gloo host tests).  If the library's communicator cannot be created
    (its RCCL is the image's /opt/rocm one, torch.distributed's is torch's own build), the
    same collectives run through torch.distributed's process group -- RCCL on the GPU as
    well, not a host path -- and the switch is reported on stderr."""
    if world_size == 1:
        return LocalComm()
    if device.type != "cuda" or os.environ.get("HDP_COMM", "rccl") == "torch":
        return TorchComm(rank, world_size, group)
    try:
        return RcclComm(rank, world_size, group)
    except Exception as e:  # noqa: BLE001 -- any init failure: the torch.distributed collectives instead
        print(f"hdpissa: rank {rank}: the library's RCCL communicator failed ({e}); "
              "using torch.distributed collectives (HDP_COMM=torch)", file=sys.stderr, flush=True)
        return TorchComm(rank, world_size, group)
