"""Learning-rate schedule of the reference training loop (host scalar math, hp:302-307, 338-344)."""
from __future__ import annotations

import math


def total_steps(num_epochs: int, len_dataloader: int, accumulation_steps: int) -> int:
    """hp:305 (accumulation_steps is already divided by world_size, hp:266)."""
    return num_epochs * len_dataloader // accumulation_steps


def warmup_steps_from(warmup_steps: int, warmup_ratio: float, total: int) -> int:
    """hp:306-307."""
    if warmup_steps == 0 and warmup_ratio > 0:
        return int(warmup_ratio * total)
    return warmup_steps


def lr_at(t: int, initial_lr: float, warmup_steps: int, total: int, schedule: str = "cosine") -> float:
    """LR of the optimizer step whose counter is ``t`` *before* the increment (hp:338-344).
    The first step after a warmup start uses t = 0, i.e. lr = 0 (a no-op update)."""
    if t < warmup_steps:
        return initial_lr * t / warmup_steps
    if schedule == "cosine":
        return 0.5 * initial_lr * (1 + math.cos(math.pi * (t - warmup_steps) / (total - warmup_steps)))
    return initial_lr * (1 - (t - warmup_steps) / (total - warmup_steps))
