"""Checkpoint export (hp:46-79): the merged weight of every adapter layer IS its W_res."""
from __future__ import annotations

import os

import torch
import torch.nn as nn

from .layer import CustomLinearLayer, _bind_residual_factors, get_parent_module


def save_custom_model(model: nn.Module, tokenizer, model_path: str) -> None:
    """Temporarily swap every CustomLinearLayer for an nn.Linear holding W_res, call
    ``save_pretrained`` on the model (and tokenizer, if given), then restore (hp:46-79)."""
    os.makedirs(model_path, exist_ok=True)
    saved = {n: m for n, m in model.named_modules() if isinstance(m, CustomLinearLayer)}
    for name, layer in saved.items():
        new = nn.Linear(layer.in_features, layer.out_features, bias=layer.bias is not None, device="meta")
        new.weight = nn.Parameter(layer.merge_weights(), requires_grad=False)
        new.bias = layer.bias
        setattr(get_parent_module(model, name), name.split(".")[-1], new)
    try:
        target = model.module if isinstance(model, torch.nn.parallel.DistributedDataParallel) else model
        target.save_pretrained(model_path)
        if tokenizer is not None:
            tokenizer.save_pretrained(model_path)
    finally:
        for name, layer in saved.items():
            setattr(get_parent_module(model, name), name.split(".")[-1], layer)


def export_merged_safetensors(model: nn.Module, path: str) -> None:
    """Write only the merged adapter weights (W_res) as safetensors, keyed '<module>.weight'."""
    from safetensors.torch import save_file
    tensors = {f"{n}.weight": m.merge_weights().contiguous().cpu()
               for n, m in model.named_modules() if isinstance(m, CustomLinearLayer)}
    save_file(tensors, path)


# -- resume state (absent in the reference: its Adam moments and t live only in memory, hp:290-300) --
def _arenas(model: nn.Module):
    seen, out = set(), []
    for n, m in model.named_modules():
        if isinstance(m, CustomLinearLayer) and m._arena is not None and id(m._arena) not in seen:
            seen.add(id(m._arena))
            out.append(m._arena)
    return out


def save_hdpissa_state(model: nn.Module, path: str, t: int) -> None:
    """Everything an HD-PiSSA run needs to resume at an optimizer-step boundary, one safetensors
    file per rank: every rank's factors (fac_all: A, B are frozen after init, hp:375-376), this
    rank's Adam moments m, v and pending gradients, the merged weights W_res (they change every
    step, hp:394) and the step counter t (hp:300, 350).  Metadata records the module layout
    (names, shapes, r, arena offsets, and whether the layer stores the PiSSA residual -- there
    W_res = W - sum B_i A_i, so the same W_res means a different effective weight) so
    load_hdpissa_state refuses a mismatched model."""
    import json
    from safetensors.torch import save_file
    names = {id(m): n for n, m in model.named_modules()}
    tensors, meta = {}, {"t": str(int(t)), "format": "hdpissa-resume-1"}
    layout = []
    for ai, a in enumerate(_arenas(model)):
        for k in ("fac_all", "m", "v", "grad"):
            tensors[f"arena{ai}.{k}"] = getattr(a, k).detach().contiguous().cpu()
        mods = []
        for L, (oa, ob) in zip(a.layers, a.offsets):
            n = names[id(L)]
            tensors[f"{n}.W_res"] = L.W_res.detach().contiguous().cpu()
            mods.append([n, L.out_features, L.in_features, L.r, oa, ob, bool(L.residual)])
        layout.append({"world_size": a.world_size, "rank": a.rank, "F": a.F, "modules": mods})
    meta["layout"] = json.dumps(layout)
    save_file(tensors, path, metadata=meta)


def load_hdpissa_state(model: nn.Module, path: str) -> int:
    """Restore save_hdpissa_state's file into the model's arenas and W_res buffers in place
    (views stay valid: layer.A / B / m_A ... keep pointing at the arena; residual-mode layers
    rebuild their frozen-component copies from the restored factors).  Returns t."""
    import json
    from safetensors import safe_open
    names = {id(m): n for n, m in model.named_modules()}
    with safe_open(path, framework="pt") as f:
        meta = f.metadata()
        if meta.get("format") != "hdpissa-resume-1":
            raise ValueError(f"{path}: not an HD-PiSSA resume file")
        layout = json.loads(meta["layout"])
        arenas = _arenas(model)
        if len(layout) != len(arenas):
            raise ValueError("resume file and model have different adapter arenas")
        for ai, (a, lay) in enumerate(zip(arenas, layout)):
            mods = [[names[id(L)], L.out_features, L.in_features, L.r, oa, ob, bool(L.residual)]
                    for L, (oa, ob) in zip(a.layers, a.offsets)]
            saved = [m if len(m) == 7 else m + [False] for m in lay["modules"]]  # files before the flag
            if lay["world_size"] != a.world_size or lay["rank"] != a.rank or lay["F"] != a.F or saved != mods:
                raise ValueError("resume file layout does not match the model (modules, shapes, r, world size, "
                                 "rank or residual mode)")
            with torch.no_grad():
                for k in ("fac_all", "m", "v", "grad"):
                    getattr(a, k).copy_(f.get_tensor(f"arena{ai}.{k}"))
                for L in a.layers:
                    L.W_res.copy_(f.get_tensor(f"{names[id(L)]}.W_res"))
                    if L.residual:  # the forward's x A_all^T B_cat^T must use the restored factors
                        _bind_residual_factors(L)
        return int(meta["t"])
