"""The HD-PiSSA optimizer step: hp:352-398 on MI355X.

Reference, per module per step: ~20 elementwise launches of Adam, 4 all_gathers (dA, dB and
the *constant* A, B), 4*Wn zeros_like, Wn x (3 GEMMs + 3 elementwise over out x in) and a
merge -- ~48 N Wn bytes of HBM traffic per rank.  Here, per arena (all modules):

  1. K3  one Adam launch over the flat arena: grad (x1e16) -> m, v -> delta; clears grad.
         (Wn = 1 with single-segment H2 plans -- bf16 W, r >= 32: Adam runs inside the plan's operand
         preparation instead, writing the delta halves of the fp16 panels as it goes)
  2. exchange -- two interchangeable strategies (``exchange=``):
     "gather"    (default) RCCL all-gather of the deltas only (A_i, B_i were shared at
                 init), bucketed on a side stream; per module ONE fused K4 launch with
                 K = 2 r Wn that recomputes sum_i (B'_i A'_i - B_i A_i) in the reference's
                 rank order and merges it into W_res in the epilogue (dW never hits HBM).
     "allreduce" (north-star contract) per module K4 with K = 2r writes this rank's dW_i into
                 a bucketed float32 buffer; RCCL all-reduce of each bucket on a side stream,
                 overlapped with the next bucket's K4; then the K5 merge kernel W += sum dW.
                 bf16 models: the same buckets exchanged rank-ordered (all-to-all of the float32
                 terms, bf16 fold in rank order, all-gather of the bf16 shards, K5), which is the
                 reference's per-rank bf16 rounding (hp:389-392) that a summing all-reduce loses.
  3. A.grad = B.grad = None  (hp:397-398).

Semantics kept from the reference: Adam without weight decay, bias correction with the
post-increment t (hp:350), A and B never updated (hp:375-376; the deltas are recomputed
against the *initial* factors every step), grads scaled x1e16 (hp:356-357), bf16 models
accumulate dW in bf16 rank by rank (zeros_like(W_res), hp:389).
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn as nn

from ._lib import HDP_DW_MERGE, HDP_DW_STORE
from .layer import CustomLinearLayer, FactorArena, custom_layers


def _buckets(sizes: List[int], cap: int) -> List[Tuple[int, int]]:
    """Greedy contiguous buckets of module indices with sum(size) <= cap (>= 1 module each)."""
    out, start, acc = [], 0, 0
    for i, s in enumerate(sizes):
        if acc and acc + s > cap:
            out.append((start, i))
            start, acc = i, 0
        acc += s
    if start < len(sizes):
        out.append((start, len(sizes)))
    return out


class _ArenaPlan:
    def __init__(self, arena: FactorArena, exchange: str, bucket_bytes: int):
        self.arena = arena
        Wn, F = arena.world_size, arena.F
        dev = arena.fac.device
        n = len(arena.layers)
        # gather: buckets over the delta arena (module-aligned ranges)
        ends = [arena.offsets[i + 1][0] if i + 1 < n else F for i in range(n)]
        starts = [arena.offsets[i][0] for i in range(n)]
        self.g_buckets = []
        for a, b in _buckets([ends[i] - starts[i] for i in range(n)], max(1, bucket_bytes // 4 // max(Wn, 1))):
            self.g_buckets.append((a, b, starts[a], ends[b - 1]))
        self.delta_all = torch.empty(Wn * F, dtype=torch.float32, device=dev) if (exchange == "gather" and Wn > 1) else None
        # allreduce: buckets over dense dW sizes
        self.a_buckets = []
        self.dw_bufs: List[torch.Tensor] = []
        # rank-ordered bf16 exchange (bf16 buckets at Wn > 1): per bucket the 1/Wn shard length (a
        # multiple of 8 elements), the all-to-all receive buffers, the folded bf16 shards and the
        # all-gathered bf16 dW (double-buffered like dw_bufs)
        self.a_ordered: List[bool] = []
        self.a_shard: List[int] = []
        self.o_recv: List[torch.Tensor] = []
        self.o_shard: List[torch.Tensor] = []
        self.o_gath: List[torch.Tensor] = []
        if exchange == "allreduce":
            sizes = [L.out_features * L.in_features for L in arena.layers]
            self.a_buckets = _buckets(sizes, max(1, bucket_bytes // 4))
            cap = max(sum(sizes[a:b]) for a, b in self.a_buckets)
            for a, b in self.a_buckets:
                n = sum(sizes[a:b])
                self.a_ordered.append(Wn > 1 and all(arena.layers[i].W_res.dtype == torch.bfloat16 for i in range(a, b)))
                self.a_shard.append(-(-n // (8 * Wn)) * 8)
            if any(self.a_ordered):
                sh = max(s for s, o in zip(self.a_shard, self.a_ordered) if o)
                cap = max(cap, Wn * sh)
                self.o_recv = [torch.empty(Wn * sh, dtype=torch.float32, device=dev) for _ in range(2)]
                self.o_shard = [torch.empty(sh, dtype=torch.bfloat16, device=dev) for _ in range(2)]
                self.o_gath = [torch.empty(Wn * sh, dtype=torch.bfloat16, device=dev) for _ in range(2)]
            self.dw_bufs = [torch.zeros(cap, dtype=torch.float32, device=dev) for _ in range(2)]
        self.plans: Dict[tuple, list] = {}   # grouped K4 launches, built on first use

    def delta_plans(self, key, ops, make_items, mode, dsts) -> list:
        """Grouped K4 plans for one launch site (cached; rebuilt if a destination moved).
        Items are split where the destination dtype changes (one plan per dtype run)."""
        plans = self.plans.get(key)
        if plans is not None:
            ok, k = True, 0
            for p, _ in plans:
                ok = ok and p.valid(dsts[k:k + p.n])
                k += p.n
            if ok and k == len(dsts):
                return plans
        items = make_items()
        plans, run = [], []
        for it, d in zip(items, dsts):
            if run and run[-1][1].dtype != d.dtype:
                plans.append(self._make_plan(ops, run, mode))
                run = []
            run.append((it, d))
        if run:
            plans.append(self._make_plan(ops, run, mode))
        self.plans[key] = plans
        return plans

    @staticmethod
    def _make_plan(ops, run, mode):
        rnd = run[0][1].dtype == torch.bfloat16
        return ops.delta_plan([it for it, _ in run], mode, rnd), [d for _, d in run]


class HDPissaStep:
    """Stateful step object: holds the exchange plan, bucket buffers, side stream and events."""

    def __init__(self, model: nn.Module, world_size: int, rank: int = 0, comm=None, ops=None,
                 exchange: str = "gather", bucket_bytes: Optional[int] = None, beta1: float = 0.9,
                 beta2: float = 0.999, eps: float = 1e-8):
        if exchange not in ("gather", "allreduce"):
            raise ValueError("exchange must be 'gather' or 'allreduce'")
        self.layers = [m for _, m in custom_layers(model)]
        if not self.layers:
            raise ValueError("model has no CustomLinearLayer")
        self.world_size, self.rank = world_size, rank
        self.exchange = exchange
        self.beta1, self.beta2, self.eps = beta1, beta2, eps
        if bucket_bytes is None:
            # gather: ~256 MB of per-rank deltas per all-gather bucket; allreduce: 1 GB of dense
            # float32 dW per bucket (two buffers): bigger K4-store / K5 launches, fewer collectives
            bucket_bytes = (256 << 20) if exchange == "gather" else (1 << 30)
        arenas: Dict[int, FactorArena] = {}
        for L in self.layers:
            if L._arena is None:
                raise RuntimeError(f"{L.name} has no factor arena")
            if L._arena.world_size != world_size:
                raise ValueError("layer world_size differs from the step's world_size")
            arenas.setdefault(id(L._arena), L._arena)
        self.plans = [_ArenaPlan(a, exchange, bucket_bytes) for a in arenas.values()]
        self.device = self.layers[0].W_res.device
        if ops is None:
            from .ops import default_ops
            ops = default_ops()
        self.ops = ops
        if comm is None:  # the arena's init communicator (module-sharded SVD) if it has one
            comm = next((p.arena.comm for p in self.plans if getattr(p.arena, "comm", None) is not None), None)
        if comm is None:
            from .comm import make_comm
            comm = make_comm(rank, world_size, self.device)
        self.comm = comm
        self.on_gpu = self.device.type == "cuda"
        self.side = torch.cuda.Stream(device=self.device) if self.on_gpu else None
        # grouped persistent K4 (one launch per bucket); HDP_DELTA_GROUPED=0 -> one launch per module
        self.grouped = hasattr(ops, "delta_plan") and os.environ.get("HDP_DELTA_GROUPED", "1") != "0"
        # K = 2 r Wn > 32 (gathered segments): the grouped plan runs the packed bf16x3 kernel
        # (tools/delta_bench.py, 56 LLaMA-7B modules: Wn 2 / 4 / 8 = 2.8 / 3.8 / 6.3 ms vs
        # 3.7 / 5.3 / 8.5 ms for per-module f32 launches)
        self.grouped_multiseg = self.grouped
        self._fuse_adam = os.environ.get("HDP_FUSED_ADAM", "1") != "0"

    def invalidate_factors(self) -> None:
        """The factors A / B were rewritten in place in a way the arena's version counter does not see
        (``.data`` writes, raw-pointer copies): every cached K4 plan re-packs its constant operand halves
        and factor maxima on its next fused Adam run.  Writes through the tensors themselves (``copy_``,
        ``load_state_dict``, ``load_hdpissa_state``) are detected without this call."""
        for plan in self.plans:
            plan.arena.probe_queue.flush()  # pending probe groups read the old operands
            for plans in plan.plans.values():
                for p, _ in plans:
                    inv = getattr(p, "invalidate", None)
                    if inv is not None:
                        inv()
        for L in self.layers:  # the probe's cached B^T and the native one-call slot captured the old B
            L._Bt = None
            L._fslot = None

    # -----------------------------------------------------------------------------------
    def _collect_grads(self, arena: FactorArena) -> None:
        """Make sure the arena's grad buffer holds every layer's A.grad / B.grad."""
        for L in arena.layers:
            prm = L._parameters  # (not nn.Module.__getattr__: 2 lookups per layer per step)
            for p, view in ((prm["A"], L._gA), (prm["B"], L._gB)):
                g = p.grad
                if g is None:
                    view.zero_()  # no backward reached this layer: zero gradient
                elif g is not view and g.data_ptr() != view.data_ptr():
                    view.copy_(g)

    def step(self, lr: float, t: int) -> None:
        """One optimizer step (hp:352-398); ``t`` is the counter after hp:350's increment."""
        with torch.no_grad():
            for plan in self.plans:
                plan.arena.probe_queue.flush()  # grads of deferred probe launches first
            chk = getattr(self.ops, "probe_errors", None)
            if chk is not None and chk():
                # a probe launch that has completed reported a failed hand-off: its gradients are
                # wrong, so no update is applied (host-mapped word: no synchronisation here).  Launches
                # still running when this check passes are covered on the device: K3 reads the same
                # word in stream order and, while it is set, leaves m / v as they were and writes
                # delta = 0, so the merge adds exactly 0 to W_res (the next flush / step raises)
                from ._lib import HdpError
                raise HdpError("probe kernels reported a failed hand-off (hdp_probe_errors); the "
                               "accumulated gradients are not trustworthy -- step refused")
            for plan in self.plans:
                self._step_arena(plan, lr, t)
        for L in self.layers:  # hp:397-398
            prm = L._parameters
            prm["A"].grad = None
            prm["B"].grad = None

    def _step_arena(self, plan: _ArenaPlan, lr: float, t: int) -> None:
        arena, ops, Wn = plan.arena, self.ops, self.world_size
        self._collect_grads(arena)
        fused = self._fused_plans(plan, lr, t)
        if fused is not None:
            # K3 folded into K4's operand preparation -- per plan one Adam pass that also
            # writes the delta halves of the H2 panels, then the merge (no standalone Adam / pack)
            for p, _ in fused:
                p.run_adam(arena.grad, arena.m, arena.v, arena.delta, t, lr, self.beta1, self.beta2, self.eps,
                           zero_grad=True)
            return
        ops.adam(arena.grad, arena.m, arena.v, arena.delta, t, lr, self.beta1, self.beta2, self.eps, zero_grad=True)
        if self.exchange == "gather":
            self._gather(plan)
        else:
            self._allreduce(plan)

    def _fused_plans(self, plan: _ArenaPlan, lr: float, t: int):
        """The Wn = 1 gather plans when every one of them folds Adam in (single-segment H2 merges:
        bf16 W at r >= 32), else None (HDP_FUSED_ADAM=0 turns the fold off)."""
        if not (self.exchange == "gather" and self.world_size == 1 and self.grouped) or not self._fuse_adam:
            return None
        from .ops import adam_delta_bound
        if adam_delta_bound(t, lr, self.beta1, self.beta2) is None:
            return None
        arena = plan.arena
        plans = plan.delta_plans("g1", self.ops, lambda: self._items_w1(arena), HDP_DW_MERGE,
                                 [L.W_res for L in arena.layers])
        if all(getattr(p, "fused_adam", None) is not None and p.fused_adam() for p, _ in plans):
            return plans
        return None

    @staticmethod
    def _items_w1(arena: FactorArena):
        out = []
        for i, L in enumerate(arena.layers):
            oa, ob = arena.offsets[i]
            out.append((L.out_features, L.in_features, L.r, 1, arena.delta[oa:], arena.delta[ob:], 0,
                        arena.fac[oa:], arena.fac[ob:], 0, L.W_res))
        return out

    # -- exchange = "gather" -------------------------------------------------------------
    def _gather(self, plan: _ArenaPlan) -> None:
        arena, ops, Wn, F = plan.arena, self.ops, self.world_size, plan.arena.F
        if Wn == 1:
            if self.grouped:
                for p, _ in plan.delta_plans("g1", ops, lambda: self._items_w1(arena), HDP_DW_MERGE,
                                             [L.W_res for L in arena.layers]):
                    p.run()
                return
            for it in self._items_w1(arena):
                ops.delta_gemm(*it, HDP_DW_MERGE, it[-1].dtype == torch.bfloat16)
            return
        cur = torch.cuda.current_stream(self.device) if self.on_gpu else None
        events = []
        if self.on_gpu:
            ready = torch.cuda.Event()
            ready.record(cur)
            with torch.cuda.stream(self.side):
                self.side.wait_event(ready)
                for (a, b, s, e) in plan.g_buckets:
                    self.comm.allgather(arena.delta[s:e], plan.delta_all[Wn * s:Wn * e])
                    ev = torch.cuda.Event()
                    ev.record(self.side)
                    events.append(ev)
        else:
            for (a, b, s, e) in plan.g_buckets:
                self.comm.allgather(arena.delta[s:e], plan.delta_all[Wn * s:Wn * e])
        for bi, (a, b, s, e) in enumerate(plan.g_buckets):
            if self.on_gpu:
                cur.wait_event(events[bi])
            seg = e - s
            base = plan.delta_all[Wn * s:]

            def items(a=a, b=b, s=s, seg=seg, base=base):
                out = []
                for i in range(a, b):
                    L = arena.layers[i]
                    oa, ob = arena.offsets[i]
                    out.append((L.out_features, L.in_features, L.r, Wn, base[oa - s:], base[ob - s:], seg,
                                arena.fac_all.view(-1)[oa:], arena.fac_all.view(-1)[ob:], F, L.W_res))
                return out
            if self.grouped and self.grouped_multiseg:
                for p, _ in plan.delta_plans(("g", bi), ops, items, HDP_DW_MERGE,
                                             [arena.layers[i].W_res for i in range(a, b)]):
                    p.run()
                continue
            for it in items():
                ops.delta_gemm(*it, HDP_DW_MERGE, it[-1].dtype == torch.bfloat16)

    # -- exchange = "allreduce" ----------------------------------------------------------
    def _allreduce(self, plan: _ArenaPlan) -> None:
        arena, ops = plan.arena, self.ops
        cur = torch.cuda.current_stream(self.device) if self.on_gpu else None
        freed = [None, None]
        last = None
        for bi, (a, b) in enumerate(plan.a_buckets):
            buf = plan.dw_bufs[bi % 2]
            if self.on_gpu and freed[bi % 2] is not None:
                cur.wait_event(freed[bi % 2])  # the merges that read this buffer are done
            off, slots, items = 0, [], []
            for i in range(a, b):
                L = arena.layers[i]
                oa, ob = arena.offsets[i]
                n = L.out_features * L.in_features
                items.append((L.out_features, L.in_features, L.r, 1, arena.delta[oa:], arena.delta[ob:], 0,
                              arena.fac[oa:], arena.fac[ob:], 0, buf[off:off + n]))
                slots.append((L, off, n))
                off += n
            if self.grouped:
                for p, _ in plan.delta_plans(("a", bi), ops, lambda items=items: items, HDP_DW_STORE,
                                             [it[-1] for it in items]):
                    p.run()
            else:
                for it in items:
                    ops.delta_gemm(*it, HDP_DW_STORE, False)
            if self.on_gpu and self.world_size == 1:
                # the all-reduce of one rank is the identity: the bucket's K5 follows its K4 on the
                # same stream (a side-stream merge would only contend with the next K4 for HBM)
                ops.merge_group([(L.W_res, buf[o:o + n].view_as(L.W_res)) for L, o, n in slots])
            elif self.on_gpu:
                computed = torch.cuda.Event()
                computed.record(cur)
                with torch.cuda.stream(self.side):
                    self.side.wait_event(computed)
                    self._exchange_merge(plan, bi, buf, off, slots)
                    ev = torch.cuda.Event()
                    ev.record(self.side)
                freed[bi % 2] = ev
                last = ev
            else:
                self._exchange_merge(plan, bi, buf, off, slots)
        if self.on_gpu and last is not None:
            cur.wait_event(last)


    def _exchange_merge(self, plan: _ArenaPlan, bi: int, buf: torch.Tensor, off: int, slots) -> None:
        """One bucket's exchange + merge on the current stream.

        float32 W: RCCL all-reduce of the per-rank float32 dW_i, then K5 (W += sum_i dW_i).
        bfloat16 W (rank-ordered): the reference rounds its running dW to bf16 after EVERY rank's
        term, in rank order (hp:389-392: zeros_like(W_res) is bf16), which a summing all-reduce
        cannot reproduce.  Instead an all-to-all hands every rank all Wn float32 terms of its 1/Wn
        shard of the bucket, the fold kernel applies them in rank order with the bf16 rounding
        (hdp_fold_bf16), the folded bf16 shards are all-gathered, and K5 merges bf16(W + dW) --
        the reference's arithmetic, on 6 N (Wn - 1) / Wn bytes per rank instead of the ring
        all-reduce's 8 N (Wn - 1) / Wn."""
        ops, Wn = self.ops, self.world_size
        if plan.a_ordered and plan.a_ordered[bi]:
            sh = plan.a_shard[bi]
            k = bi % 2
            recv, shard, gath = plan.o_recv[k][:Wn * sh], plan.o_shard[k][:sh], plan.o_gath[k][:Wn * sh]
            self.comm.alltoall(buf[:Wn * sh], recv)
            ops.fold_bf16(recv.view(Wn, sh), shard)
            self.comm.allgather_any(shard, gath)
            src = gath
        else:
            self.comm.allreduce_sum(buf[:off])
            src = buf
        if hasattr(ops, "merge_group"):  # the bucket's K5 as one launch
            ops.merge_group([(L.W_res, src[o:o + n].view_as(L.W_res)) for L, o, n in slots])
        else:
            for L, o, n in slots:
                ops.merge(L.W_res, src[o:o + n])


_STEPPERS: Dict[int, HDPissaStep] = {}


def hd_pissa_step(model: nn.Module, lr: float, t: int, world_size: int, rank: int = 0, beta1: float = 0.9,
                  beta2: float = 0.999, epsilon: float = 1e-8, exchange: str = "gather", comm=None,
                  ops=None) -> HDPissaStep:
    """Functional form of the reference block hp:352-398 (one call per optimizer step).
    The step object (plan, buffers, streams) is cached per model."""
    st = _STEPPERS.get(id(model))
    if st is None or st.exchange != exchange:
        st = HDPissaStep(model, world_size, rank, comm=comm, ops=ops, exchange=exchange, beta1=beta1, beta2=beta2,
                         eps=epsilon)
        _STEPPERS[id(model)] = st
    st.step(lr, t)
    return st
