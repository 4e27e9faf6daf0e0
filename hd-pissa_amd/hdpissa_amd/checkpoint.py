"""Checkpoint export (hp:46-79): the merged weight of every adapter layer IS its W_res."""
from __future__ import annotations

import os

import torch
import torch.nn as nn

from .layer import CustomLinearLayer, get_parent_module


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
    tensors = {f"{n}.weight": m.W_res.detach().contiguous().cpu()
               for n, m in model.named_modules() if isinstance(m, CustomLinearLayer)}
    save_file(tensors, path)
