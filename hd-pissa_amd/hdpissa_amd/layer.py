"""Drop-in adapter layer: ``CustomLinearLayer`` and ``replace_with_custom_layer``.

Mirrors the reference API (hd_pissa.py, "hp:") attribute for attribute:
  CustomLinearLayer(original_linear, name, device_id, world_size, ranks_per_gpu=None,
                    alpha=0.0, dropout=0.0)                                  hp:95-134
    .name .in_features .out_features .dropout_rate .dropout .alpha (= alpha // r)
    .A (r x in, float32 Parameter)  .B (out x r, float32 Parameter)
    .W_res (buffer, model dtype, = the pretrained W -- hp:129)  .bias
    forward(x) -> model dtype                                                hp:136-140
    merge_weights() -> W_res.clone()                                         hp:142-144
  replace_with_custom_layer(model, target_modules, rank, world_size, ranks_per_gpu=None,
                            alpha=0.0, dropout=0.0)                          hp:150-156
  get_parent_module(model, name)                                             hp:81-86

What changes underneath (MI355X-native):
  * init (K1): top r*world_size triplets only (fp64 Gram + rocSOLVER + projection), and with
    a process group the SVDs are sharded round-robin over ranks and broadcast once -- every
    rank then holds every rank's (A_i, B_i), which the gather exchange needs (the reference
    re-gathers these constants every step, hp:386-387);
  * forward = the base linear (hipBLASLt through torch); the 1e-16-scaled adapter term of
    hp:139 is below float32 resolution of the output and is not formed;
  * backward: the probe gradients come from skinny fp32-MFMA kernels (K2) written straight
    into a flat factor arena that the step's single Adam launch (K3) and the all-gather
    consume; A.grad / B.grad are views of that arena with the reference's 1e-16 scale.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import os

import numpy as np

import torch
import torch.nn as nn
import torch.nn.functional as F

ALIGN = 64  # float elements: every factor block starts 256-byte aligned in the arena


def get_parent_module(model: nn.Module, module_name: str) -> nn.Module:
    """hp:81-86."""
    parent = model
    for part in module_name.split(".")[:-1]:
        parent = getattr(parent, part)
    return parent


def _alpha_eff(alpha, ranks_per_gpu):
    if ranks_per_gpu is None:
        # hp:103 evaluates `alpha // ranks_per_gpu` before the None default at hp:112-113
        raise TypeError("ranks_per_gpu=None: the reference fails here too (hp:103 runs before hp:112)")
    return alpha // ranks_per_gpu


def _round_up(n: int, a: int = ALIGN) -> int:
    return (n + a - 1) // a * a


class FactorArena:
    """Flat float32 storage for a group of adapter layers, laid out per module as
    [A (r x in) | B (out x r)] at 256-byte aligned offsets:

      fac   [F]          this rank's factors; layer.A / layer.B are views
      grad  [F]          probe gradients (reference scale); layer.A.grad / .B.grad are views
      m, v  [F]          Adam moments (layer.m_A ... are views, hp:290-295)
      delta [F]          this step's (dA, dB)
      fac_all [Wn, F]    every rank's factors (constant; gathered once at init)
    """

    def __init__(self, layers: List["CustomLinearLayer"], factors_all: List[Tuple[torch.Tensor, torch.Tensor]],
                 world_size: int, rank: int, device):
        self.layers = layers
        self.world_size, self.rank = world_size, rank
        self.offsets: List[Tuple[int, int]] = []
        off = 0
        for L in layers:
            oa = off
            ob = oa + _round_up(L.r * L.in_features)
            off = ob + _round_up(L.out_features * L.r)
            self.offsets.append((oa, ob))
        self.F = off
        kw = dict(dtype=torch.float32, device=device)
        self.fac_all = torch.zeros(world_size, self.F, **kw)
        self.fac = self.fac_all[rank]
        self.grad = torch.zeros(self.F, **kw)
        self.m = torch.zeros(self.F, **kw)
        self.v = torch.zeros(self.F, **kw)
        self.delta = torch.zeros(self.F, **kw)
        for L, (oa, ob), (A_all, B_all) in zip(layers, self.offsets, factors_all):
            r, inn, out = L.r, L.in_features, L.out_features
            for i in range(world_size):
                self.fac_all[i, oa:oa + r * inn].view(r, inn).copy_(A_all[i * r:(i + 1) * r])
                self.fac_all[i, ob:ob + out * r].view(out, r).copy_(B_all[i])
            L._bind(self, oa, ob)
        self.probe_queue = ProbeQueue(layers[0].ops if layers else None)
        self.comm = None  # the communicator of the sharded init, if any (replace_with_custom_layer)

    def views(self, buf: torch.Tensor, idx: int):
        L = self.layers[idx]
        oa, ob = self.offsets[idx]
        return (buf[oa:oa + L.r * L.in_features].view(L.r, L.in_features),
                buf[ob:ob + L.out_features * L.r].view(L.out_features, L.r))


def _raw_stream(device) -> int:
    return torch._C._cuda_getCurrentRawStream(device.index if device.index is not None else torch.cuda.current_device())


class ProbeQueue:
    """Deferred, grouped probe backward (K2) for the layers of one arena.

    ``CustomLinearLayer._probe_backward`` enqueues (X, G); the queue launches one grouped
    kernel set per flush.  Flushes happen (a) when autograd finishes the current backward
    pass (engine callback), so ``A.grad`` / ``B.grad`` are complete when ``backward()``
    returns, exactly as in the reference; (b) before a layer would appear twice in a group;
    (c) at ``max_group`` items (256; env HDP_PROBE_GROUP) or when ``budget`` bytes of pending X+G
    would be exceeded (default 16 GB, env HDP_PROBE_BUDGET_MB): a whole backward pass is normally ONE
    group -- each sweep phase launch has a ramp and a tail of ~10-15 us whatever its size, so the
    six launches of a group are amortised over every module of the pass; (d) at the start of every
    optimizer step.  The queue holds X and G
    alive until the flush has enqueued the kernels on the stream that produced them.

    Host path: on a HIP device with the library's op set, the queue is the NATIVE
    ``hdp_probe_queue`` (include/hdpissa.h) behind its torch binding ``hdpissa_amd._C.ProbeQueue``
    (hd-pissa_amd/csrc_ext): every layer registers its constant operands once (a slot per layer
    and X dtype) and each module backward is ONE native call pushing (slot, X, G, accumulate) on
    the current stream; the binding keeps the pushed X / G alive until their group is launched
    and the queue forms and launches the groups.  (Through Python + ctypes the push cost ~11 us
    of host time per module backward -- the bench's probe phase was host-bound.)  Other op sets
    (the CPU test ops) and gradients that are not the arena views take the Python path below.
    """

    def __init__(self, ops, budget_bytes: Optional[int] = None):
        self.ops = ops
        if budget_bytes is None:
            budget_bytes = int(float(os.environ.get("HDP_PROBE_BUDGET_MB", "16384")) * (1 << 20))
        self.budget = budget_bytes
        self.items = []     # (layer, X, G, gA, gB, scale, accumulate)
        self.layers = set()
        self.bytes = 0
        self.ws_bytes = 0
        self.stream = None
        self._cb_task = -1
        self._max = None
        self._fast = hasattr(ops, "probe_group_raw")
        self._carr = None
        self._nq = {}             # x dtype -> native queue (hdpissa_amd._C.ProbeQueue)
        self._native_dtype = None  # dtype of the native queue holding pending modules, if any
        self._nmax = int(os.environ.get("HDP_PROBE_GROUP", "256"))

    def _max_group(self) -> int:
        if self._max is None:
            f = getattr(self.ops, "probe_group_max", None)
            self._max = f() if f is not None else 16
            if self._fast:
                from ._lib import ProbeItem
                self._carr = (ProbeItem * self._max)()
        return self._max

    # -- native path -----------------------------------------------------------------------
    def _native_queue(self, dtype):
        q = self._nq.get(dtype)
        if q is None:
            from . import _C
            q = self._nq[dtype] = _C.ProbeQueue(dtype == torch.bfloat16, min(self._nmax, self._max_group()),
                                                self.budget)
            if len(self._nq) > 1:  # a second dtype: every push through push_native (keeps push order)
                for other in self._nq.values():
                    other.set_fast(False)
        return q

    def push_native(self, layer, x, gy, accumulate) -> None:
        """One module backward onto the native queue (x: [..., in], gy: [..., out])."""
        dt = x.dtype
        for odt, oq in self._nq.items():
            if odt is not dt and oq.pending():
                # one native queue per X dtype: launch the other queue's pending group first, so
                # groups run in push order (an overwrite never overtakes an earlier accumulate)
                self._flush_native()
                break
        q = self._nq.get(dt)
        if q is None:
            q = self._native_queue(dt)
        ent = layer._nslot.get(dt)
        if ent is None or ent[1] is not layer.A or ent[2] is not layer._Bt or layer.B._version != layer._Bt_version:
            if ent is not None:  # re-registration (A replaced / B edited): the pending group reads the old operands
                self._flush_native()
            layer._fslot = None
            Bt = layer._b_transposed()
            slot = q.add_module(layer.A.data_ptr(), Bt.data_ptr(), layer._gA.data_ptr(), layer._gB.data_ptr(),
                                layer.in_features, layer.out_features, layer.r, layer._scale)
            ent = layer._nslot[dt] = (slot, layer.A, Bt)
        q.push(ent[0], x, gy, accumulate, layer.in_features, layer.out_features)
        self._native_dtype = dt
        if len(self._nq) == 1 and layer._fslot is None:
            # from now on this layer's module backward is one native call (LayerSlot.push)
            from . import _C
            layer._fslot = _C.LayerSlot(q, ent[0], layer.A, layer.B, layer._gA, layer._gB, layer.in_features,
                                        layer.out_features, layer._Bt_version)
        task = torch._C._current_graph_task_id()  # -1 outside a backward pass (0.1 us)
        if task != -1 and task != self._cb_task:
            torch.autograd.Variable._execution_engine.queue_callback(self._end_of_backward)
            self._cb_task = task

    def _flush_native(self) -> None:
        # every native queue (a layer's LayerSlot pushes without passing through Python); a flush
        # of an empty queue returns at once
        for q in self._nq.values():
            try:
                q.flush()
            except RuntimeError as e:  # the library's refusal, as the Python path reports it
                from ._lib import HdpError
                if isinstance(e, HdpError):
                    raise
                raise HdpError(str(e)) from e
        self._native_dtype = None

    def close(self) -> None:
        self._flush_native()
        for q in self._nq.values():
            q.close()
        self._nq = {}

    def __del__(self):
        try:
            if self._nq:
                self.close()
        except Exception:
            pass

    def native_ok(self, layer, x, gA, gB) -> bool:
        """The native push applies: library ops, a HIP tensor, no Python-path group pending, and
        the gradients are the layer's arena views."""
        return (self._fast and not self.items and x.is_cuda and (gA is layer._gA or gA.data_ptr() == layer._gA.data_ptr())
                and (gB is layer._gB or gB.data_ptr() == layer._gB.data_ptr()))

    def enqueue(self, layer, X, G, gA, gB, scale, accumulate) -> None:
        cuda = X.is_cuda
        if self.native_ok(layer, X, gA, gB):
            self.push_native(layer, X, G, accumulate)
            return
        self._flush_native()  # keep the launch order when a Python-path item follows native ones
        stream = _raw_stream(X.device) if cuda else None
        nb = X.numel() * X.element_size() + G.numel() * G.element_size()
        mx = self._max_group()
        if self.items and (id(layer) in self.layers or stream != self.stream or len(self.items) >= mx or
                           self.bytes + nb > self.budget or X.dtype != self.items[0][1].dtype):
            self.flush()
        if not self.items:
            self.stream = stream
        n = len(self.items)
        self.items.append((layer, X, G, gA, gB, scale, accumulate))
        self.layers.add(id(layer))
        self.bytes += nb
        if self._fast and cuda:
            self.ws_bytes += layer._fill_probe_item(self._carr, n, X, G, gA, gB, accumulate)
        task = torch._C._current_graph_task_id()  # -1 outside a backward pass (0.1 us)
        if task != -1 and task != self._cb_task:
            # flush when the running backward pass completes (once per graph task; outside a
            # backward pass the queue is flushed by budget / step / flush())
            torch.autograd.Variable._execution_engine.queue_callback(self._end_of_backward)
            self._cb_task = task

    def _end_of_backward(self) -> None:
        self.flush()

    def flush(self) -> None:
        self._flush_native()
        if not self.items:
            return
        items, stream, wsb = self.items, self.stream, self.ws_bytes
        X0 = items[0][1]
        # the group stays queued until its launch succeeds (a refused launch -- the probe error word
        # is set -- must not drop modules whose gradients would then silently go missing)
        if stream is None:
            self.ops.probe_grads_group([(X, G, L.A.detach(), L._b_transposed(), gA, gB, s, acc)
                                        for (L, X, G, gA, gB, s, acc) in items])
        elif self._fast:
            self.ops.probe_group_raw(self._carr, len(items), X0, wsb, stream)
        else:
            with torch.cuda.stream(torch.cuda.ExternalStream(stream, device=X0.device)):
                self.ops.probe_grads_group([(X, G, L.A.detach(), L._b_transposed(), gA, gB, s, acc)
                                            for (L, X, G, gA, gB, s, acc) in items])
        self.items, self.layers, self.bytes, self.ws_bytes = [], set(), 0, 0
        if stream is not None:
            # the kernels read X / G on `stream`: whatever stream allocated them, the caching allocator
            # must not hand their blocks out before that stream has passed the group (a no-op for
            # blocks allocated on `stream` itself)
            ext = torch.cuda.ExternalStream(stream, device=X0.device)
            for it in items:
                it[1].record_stream(ext)
                it[2].record_stream(ext)

    def pending(self, layer) -> bool:
        if id(layer) in self.layers:
            return True
        for dt, q in self._nq.items():
            ent = layer._nslot.get(dt)
            if ent is not None and q.pending_slot(ent[0]):
                return True
        return False


class _ProbeLinearFn(torch.autograd.Function):
    """y = x W_res^T + b; backward: dX = G W_res (when needed) and the adapter probe
    gradients accumulated by K2 into the layer's arena grad views."""

    @staticmethod
    def forward(ctx, x, W_res, bias, A, B, layer):
        ctx.save_for_backward(x)
        ctx.layer = layer
        return F.linear(x, W_res, bias)

    @staticmethod
    def backward(ctx, gy):
        (x,) = ctx.saved_tensors
        layer = ctx.layer
        dx = gy.matmul(layer.W_res) if ctx.needs_input_grad[0] else None
        layer._probe_backward(x, gy)
        return dx, None, None, None, None, None


class CustomLinearLayer(nn.Module):
    """HD-PiSSA adapter layer (hp:95-148); see the module docstring."""

    def __init__(self, original_linear: nn.Linear, name: str, device_id: int, world_size: int,
                 ranks_per_gpu: Optional[int] = None, alpha: float = 0.0, dropout: float = 0.0, *,
                 ops=None, residual: bool = False, _factors: Optional[Tuple[torch.Tensor, torch.Tensor]] = None,
                 _defer_arena: bool = False):
        super().__init__()
        self.residual = bool(residual)  # opt-in PiSSA-residual storage (see make_residual)
        self.name = name
        self.in_features = original_linear.in_features
        self.out_features = original_linear.out_features
        self.dropout_rate = dropout
        self.dropout = nn.Dropout(p=dropout)
        self.alpha = _alpha_eff(alpha, ranks_per_gpu)                        # hp:103
        if dropout and dropout > 0:
            raise NotImplementedError(
                "dropout > 0 acts elementwise on the dense out x in product B@A (hp:139), which the "
                "skinny MI355X probe path never forms; the reference configurations use dropout=0.0")
        self.r = int(ranks_per_gpu)
        self.device_id, self.world_size = device_id, world_size
        self._ops = ops
        W = original_linear.weight.data
        if _factors is None:
            _factors = self.ops.svd_topk(W, self.r, world_size)[:2]        # hp:106-125
        k = self.r * world_size
        if k > min(self.out_features, self.in_features):
            raise ValueError(f"ranks_per_gpu * world_size = {k} exceeds min(out, in) of {name}")
        A_all, B_all = _factors
        # placeholders until the arena binds the real storage
        self.A = nn.Parameter(A_all[device_id * self.r:(device_id + 1) * self.r].clone())
        self.B = nn.Parameter(B_all[device_id].clone())
        self.register_buffer("W_res", W.clone().detach())                   # hp:129 (W, not W - BA)
        self.bias = original_linear.bias if original_linear.bias is not None else None  # hp:131-134
        self._arena: Optional[FactorArena] = None
        if not _defer_arena:
            FactorArena([self], [(A_all, B_all)], world_size, device_id, W.device)
            if self.residual:
                make_residual([self])

    @property
    def ops(self):
        if self._ops is None:
            from .ops import default_ops
            self._ops = default_ops()
        return self._ops

    # -- arena binding ---------------------------------------------------------------------
    def _bind(self, arena: FactorArena, oa: int, ob: int) -> None:
        r, inn, out = self.r, self.in_features, self.out_features
        self._arena = arena
        self._oa, self._ob = oa, ob
        self.A = nn.Parameter(arena.fac[oa:oa + r * inn].view(r, inn))
        self.B = nn.Parameter(arena.fac[ob:ob + out * r].view(out, r))
        self._gA = arena.grad[oa:oa + r * inn].view(r, inn)
        self._gB = arena.grad[ob:ob + out * r].view(out, r)
        # Adam state (hp:290-295): views of the arena moments
        self._Bt, self._Bt_version = None, None
        self._tpl, self._tpl_bt, self._ws_cache = None, None, {}
        self._nslot = {}  # x dtype -> (native queue slot, A it was registered with, B^T it was registered with)
        self._fslot = None  # native one-call push of this layer's module backward (_C.LayerSlot), once registered
        self._scale = self.probe_scale
        self.m_A = arena.m[oa:oa + r * inn].view(r, inn)
        self.v_A = arena.v[oa:oa + r * inn].view(r, inn)
        self.m_B = arena.m[ob:ob + out * r].view(out, r)
        self.v_B = arena.v[ob:ob + out * r].view(out, r)

    # -- forward / backward ----------------------------------------------------------------
    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if torch.is_grad_enabled() and (self.A.requires_grad or self.B.requires_grad):
            y = _ProbeLinearFn.apply(x, self.W_res, self.bias, self.A, self.B, self)
        else:
            y = F.linear(x, self.W_res, self.bias)
        if self.residual:
            # the principal components live in the frozen factors: y += (x32 A_all^T) B_cat^T
            # (fp32, cast back like the reference's adapter term, hp:139); constant factors, so
            # autograd only carries dX through it
            y = y + F.linear(F.linear(x.float(), self._A_all), self._B_cat).to(y.dtype)
        return y

    @property
    def probe_scale(self) -> float:
        """alpha_eff * 1e-16 in float32 (hp:139's `*1e-16*self.alpha`)."""
        return float(np.float32(self.alpha) * np.float32(1e-16))

    def _probe_backward(self, x: torch.Tensor, gy: torch.Tensor) -> None:
        """Called from autograd (or directly): schedule A.grad += s (G B)^T X and
        B.grad += s G^T (X A^T) on the arena's probe queue (grouped K2 launch)."""
        fs = self._fslot
        if fs is not None and fs.push(self._parameters, x, gy):
            return  # the native push did every check below (hdp_torch_ext.cpp LayerSlot)
        q = self._arena.probe_queue
        A, B = self.A, self.B
        gA, gB = A.grad, B.grad
        if gA is None and gB is None:
            accumulate = False
            gA, gB = self._gA, self._gB
            A.grad, B.grad = gA, gB
        elif gA is not None and gB is not None:
            accumulate = True
        else:  # inconsistent user edits: start the missing one at zero
            if q.pending(self):
                q.flush()
            if gA is None:
                gA = self._gA
                gA.zero_()
                A.grad = gA
            else:
                gB = self._gB
                gB.zero_()
                B.grad = gB
            accumulate = True
        scale = self._scale
        if scale == 0.0:  # alpha // r == 0: the reference's grads are exactly zero
            if not accumulate:
                if q.pending(self):
                    q.flush()
                gA.zero_()
                gB.zero_()
            return
        if q.native_ok(self, x, gA, gB):
            # the native push takes [..., in] / [..., out] activations as they come (contiguity,
            # dtype of G and 16-byte alignment are handled there)
            q.push_native(self, x, gy, accumulate)
            return
        inn, out = self.in_features, self.out_features
        X = x if (x.dim() == 2 and x.is_contiguous()) else x.reshape(-1, inn).contiguous()
        G = gy if (gy.dim() == 2 and gy.is_contiguous()) else gy.reshape(-1, out).contiguous()
        if G.dtype != X.dtype:
            G = G.to(X.dtype)
        # the probe kernels load 16-byte row granules: a contiguous view at an odd storage
        # offset (e.g. x[1:]) is re-based into fresh storage
        if X.data_ptr() & 15:
            X = X.clone()
        if G.data_ptr() & 15:
            G = G.clone()
        q.enqueue(self, X, G, gA, gB, scale, accumulate)

    def _fill_probe_item(self, carr, n, X, G, gA, gB, accumulate) -> int:
        """Fill slot n of the queue's ctypes ProbeItem array; returns its workspace bytes."""
        import ctypes
        tpl = self._probe_item_template()
        ctypes.memmove(ctypes.byref(carr, n * ctypes.sizeof(tpl)), ctypes.byref(tpl), ctypes.sizeof(tpl))
        it = carr[n]
        it.X = X.data_ptr()
        it.G = G.data_ptr()
        T = X.shape[0]
        it.T = T
        it.accumulate = 1 if accumulate else 0
        if gA.data_ptr() != tpl.gA:
            it.gA = gA.data_ptr()
        if gB.data_ptr() != tpl.gB:
            it.gB = gB.data_ptr()
        wsb = self._ws_cache.get(T)
        if wsb is None:
            from ._lib import lib
            wsb = int(lib().hdp_probe_workspace_bytes(T, self.in_features, self.out_features, self.r))
            self._ws_cache[T] = wsb
        return wsb

    def _probe_item_template(self):
        Bt = self._b_transposed()
        if self._tpl is None or self._tpl_bt != Bt.data_ptr():
            from ._lib import ProbeItem
            t = ProbeItem()
            t.A = self.A.data_ptr()
            t.B = Bt.data_ptr()
            t.gA = self._gA.data_ptr()
            t.gB = self._gB.data_ptr()
            t.in_ = self.in_features
            t.out = self.out_features
            t.r = self.r
            t.b_transposed = 1
            t.scale = self._scale
            self._tpl, self._tpl_bt = t, Bt.data_ptr()
        return self._tpl

    def _b_transposed(self) -> torch.Tensor:
        """B^T (r x out), cached: B is frozen (hp:375-376); rebuilt if B is edited in place."""
        if self._Bt is None or self._Bt_version != self.B._version:
            self._Bt = self.B.detach().t().contiguous()
            self._Bt_version = self.B._version
        return self._Bt

    def merge_weights(self) -> torch.Tensor:
        """hp:142-144: the merged weight IS W_res (residual mode: W_res + B_cat A_all)."""
        if self.residual:
            return (self.W_res.float() + self._B_cat @ self._A_all).to(self.W_res.dtype).detach()
        return self.W_res.clone().detach()

    def __repr__(self):  # hp:146-148
        return (f"CustomLinearLayer(name={self.name}, "
                f"in_features={self.in_features}, out_features={self.out_features})")


def _find_targets(model: nn.Module, target_modules: Sequence[str]) -> List[Tuple[str, nn.Linear]]:
    """hp:151-153: substring match on named_modules(), nn.Linear only, first target wins."""
    found = []
    for name, module in model.named_modules():
        for target_name in target_modules:
            if target_name in name and isinstance(module, nn.Linear):
                found.append((name, module))
                break
    return found


def _bind_residual_factors(L: "CustomLinearLayer") -> None:
    """The frozen principal components a residual-mode layer adds back in its forward: every
    rank's factors of this module, concatenated from the arena's fac_all."""
    arena = L._arena
    i = arena.layers.index(L)
    A_all, B_all = [], []
    for d in range(arena.world_size):
        A_d, B_d = arena.views(arena.fac_all[d], i)
        A_all.append(A_d)
        B_all.append(B_d)
    L._A_all = torch.cat(A_all).contiguous()          # (Wn r) x in
    L._B_cat = torch.cat(B_all, dim=1).contiguous()   # out x (Wn r)


def make_residual(layers: Sequence["CustomLinearLayer"]) -> None:
    """Opt-in PiSSA-residual mode (north star (1); the reference keeps W_res = W, hp:129):
    W_res <- W - sum_i B_i A_i over every rank's slice (the top r*Wn components), formed on the
    device by the grouped delta GEMM (K4, MERGE mode) as  W += -sum_i [dB_i | B_i][A_i - dA_i ; dA_i]
    with dA_i := A_i (so A_i - dA_i = 0 exactly and the term is -B_i A_i).  The layer's forward adds
    the frozen components back (x A_all^T B_cat^T), merge_weights() returns W_res + B_cat A_all, and
    the HD-PiSSA update keeps flowing into W_res: the effective weight evolves exactly as in the
    default mode.  Layers must be bound to one arena."""
    if not layers:
        return
    arena = layers[0]._arena
    ops, Wn, F_ = layers[0].ops, arena.world_size, arena.F
    flat = arena.fac_all.view(-1)
    items = []
    for L in layers:
        if L._arena is not arena:
            raise ValueError("make_residual: layers of one arena only")
        i = arena.layers.index(L)
        oa, ob = arena.offsets[i]
        items.append((L.out_features, L.in_features, L.r, Wn, flat[oa:], flat[ob:], F_, flat[oa:], flat[ob:], F_,
                      L.W_res))
        _bind_residual_factors(L)
        L.residual = True
    from ._lib import HDP_DW_MERGE
    with torch.no_grad():
        for dt in {it[-1].dtype for it in items}:
            group = [it for it in items if it[-1].dtype == dt]
            if hasattr(ops, "delta_plan"):
                plan = ops.delta_plan(group, HDP_DW_MERGE, False)
                plan.run()
                if hasattr(plan, "close"):
                    plan.close()
            else:
                for it in group:
                    ops.delta_gemm(*it, HDP_DW_MERGE, False)


def replace_with_custom_layer(model: nn.Module, target_modules: Sequence[str], rank: int, world_size: int,
                              ranks_per_gpu: Optional[int] = None, alpha: float = 0.0, dropout: float = 0.0, *,
                              comm=None, ops=None, residual: bool = False) -> List[CustomLinearLayer]:
    """hp:150-156, MI355X-native.

    All targeted layers share one FactorArena.  With ``world_size > 1`` and an initialised
    torch.distributed group (or an explicit ``comm``), the top-k SVDs are sharded: module j
    is decomposed by rank ``j % world_size`` and its (A_all, B_all) broadcast to every rank.
    Returns the new layers in module order.
    """
    targets = _find_targets(model, target_modules)
    if not targets:
        return []
    _alpha_eff(alpha, ranks_per_gpu)
    r = int(ranks_per_gpu)
    if ops is None:
        from .ops import default_ops
        ops = default_ops()
    device = targets[0][1].weight.device
    if comm is None and world_size > 1 and torch.distributed.is_available() and torch.distributed.is_initialized():
        from .comm import make_comm
        comm = make_comm(rank, world_size, device)
    for name, module in targets:
        out, inn = module.out_features, module.in_features
        if r * world_size > min(out, inn):
            raise ValueError(f"ranks_per_gpu * world_size = {r * world_size} exceeds min(out, in) = "
                             f"{min(out, inn)} for {name}")
    sharded = comm is not None and world_size > 1
    # this rank's decompositions (every module, or the ones it owns when sharded), batched
    mine = [j for j in range(len(targets)) if not sharded or j % world_size == rank]
    if hasattr(ops, "svd_topk_batch"):
        done = ops.svd_topk_batch([targets[j][1].weight.data for j in mine], r, world_size)
    else:
        done = [ops.svd_topk(targets[j][1].weight.data, r, world_size) for j in mine]
    own = {j: (A_all, B_all) for j, (A_all, B_all, _) in zip(mine, done)}
    rel = getattr(ops, "release_workspace", None)
    if rel is not None:  # the batched SVD's scratch (chunks sized to HDP_SVD_BATCH_MB) is not needed after init
        rel("svd")
    factors: List[Tuple[torch.Tensor, torch.Tensor]] = []
    for j, (name, module) in enumerate(targets):
        out, inn = module.out_features, module.in_features
        if sharded:
            owner = j % world_size
            if rank == owner:
                A_all, B_all = own[j]
            else:
                A_all = torch.empty(r * world_size, inn, dtype=torch.float32, device=device)
                B_all = torch.empty(world_size, out, r, dtype=torch.float32, device=device)
            comm.broadcast(A_all, owner)
            comm.broadcast(B_all, owner)
        else:
            A_all, B_all = own[j]
        factors.append((A_all, B_all))
    layers = []
    for (name, module), fac in zip(targets, factors):
        layer = CustomLinearLayer(module, name, rank, world_size, r, alpha, dropout, ops=ops, _factors=fac,
                                  _defer_arena=True)
        setattr(get_parent_module(model, name), name.split(".")[-1], layer)
        layers.append(layer)
    arena = FactorArena(layers, factors, world_size, rank, device)
    arena.comm = comm  # reused by HDPissaStep: one communicator per process (no second RCCL comm)
    # flush_probes(model) visits these instead of walking named_modules() every call
    model.__dict__.setdefault("_hdp_arenas", []).append(arena)
    if residual:
        make_residual(layers)
    return layers


def custom_layers(model: nn.Module) -> List[Tuple[str, CustomLinearLayer]]:
    return [(n, m) for n, m in model.named_modules() if isinstance(m, CustomLinearLayer)]


def flush_probes(model: nn.Module) -> None:
    """Launch every pending grouped probe of the model's adapter layers."""
    arenas = model.__dict__.get("_hdp_arenas")
    if arenas is not None:  # the arenas replace_with_custom_layer built on this model
        for a in arenas:
            a.probe_queue.flush()
        return
    seen = set()
    for _, layer in custom_layers(model):
        a = layer._arena
        if a is not None and id(a) not in seen:
            seen.add(id(a))
            a.probe_queue.flush()


def init_adam_states(model: nn.Module) -> None:
    """hp:290-295: zero Adam moments (they live in the arena; layer.m_A ... are views)."""
    for _, layer in custom_layers(model):
        layer.m_A.zero_()
        layer.v_A.zero_()
        layer.m_B.zero_()
        layer.v_B.zero_()
