"""The training loop around the hot path (hp:297-351): micro-steps with gradient accumulation,
the learning-rate schedule, and one HD-PiSSA optimizer step (hp:352-398 -> HDPissaStep) every
``accumulation_steps`` micro-batches.

Kept from the reference: loss / accumulation_steps per micro-batch (hp:326), the schedule
evaluated at the step counter BEFORE its increment (hp:338-350), one step per accumulation
boundary ((i + 1) % accumulation_steps == 0, hp:335), the per-step loss log = the sum over the
micro-batches of the rank-averaged loss (hp:328-336).

Changed: the reference all-reduces the loss and reads it back to the host
(``.item()``) on EVERY micro-batch -- a collective and a device synchronisation per micro-step,
for logging only (the gradients do not depend on it).  Here, by default (``loss_sync="step"``),
the micro-batch losses are summed on the device in float64 and reduced / read back once per
optimizer step; ``loss_sync="micro"`` reproduces the reference's per-micro-step cadence.
"""
from __future__ import annotations

from typing import Dict, List, Optional

import torch
import torch.distributed as dist
import torch.nn as nn

from .schedule import lr_at
from .step import HDPissaStep


class HDPissaTrainer:
    def __init__(self, model: nn.Module, world_size: int, rank: int, lr: float, total_steps: int,
                 accumulation_steps: int = 1, warmup_steps: int = 0, warmup_ratio: float = 0.0,
                 schedule: str = "cosine", exchange: str = "gather", loss_sync: str = "step", comm=None, ops=None,
                 beta1: float = 0.9, beta2: float = 0.999, eps: float = 1e-8):
        if loss_sync not in ("step", "micro"):
            raise ValueError("loss_sync must be 'step' or 'micro'")
        if accumulation_steps < 1:
            raise ValueError("accumulation_steps must be >= 1 (the reference divides the global "
                             "accumulation by world_size, hp:266)")
        self.model = model
        self.world_size, self.rank = world_size, rank
        self.initial_lr = lr
        self.total_steps = total_steps
        if warmup_steps == 0 and warmup_ratio > 0:          # hp:306-307
            warmup_steps = int(warmup_ratio * total_steps)
        self.warmup_steps = warmup_steps
        self.schedule = schedule
        self.accumulation_steps = accumulation_steps
        self.loss_sync = loss_sync
        self.stepper = HDPissaStep(model, world_size, rank, comm=comm, ops=ops, exchange=exchange, beta1=beta1,
                                   beta2=beta2, eps=eps)
        self.t = 0                 # optimizer steps taken (hp:300, 350)
        self.micro = 0             # micro-batches seen in the current epoch (the reference's i)
        self.loss_list: List[float] = []
        self.lr_list: List[float] = []
        self._acc_host = 0.0       # loss_sync == "micro"
        self._acc_dev: Optional[torch.Tensor] = None  # loss_sync == "step"

    def _reduce(self, x: torch.Tensor) -> torch.Tensor:
        if self.world_size > 1 and dist.is_available() and dist.is_initialized():
            dist.all_reduce(x, op=dist.ReduceOp.SUM)
        return x

    def micro_step(self, batch: Dict[str, torch.Tensor]) -> bool:
        """One micro-batch (hp:321-333); runs the optimizer step at an accumulation boundary
        (hp:335-398).  Returns True when a step ran."""
        dev = next(self.model.parameters()).device
        input_ids = batch["input_ids"].to(dev, non_blocking=True)
        attention_mask = batch["attention_mask"].to(dev, non_blocking=True)
        labels = batch["labels"].to(dev, non_blocking=True)
        outputs = self.model(input_ids=input_ids, attention_mask=attention_mask, labels=labels)
        loss = outputs.loss / float(self.accumulation_steps)
        if self.loss_sync == "micro":
            avg = self._reduce(loss.detach().clone()) / self.world_size
            self._acc_host += avg.item()
        else:
            v = loss.detach().double()
            self._acc_dev = v if self._acc_dev is None else self._acc_dev + v
        loss.backward()
        self.micro += 1
        if self.micro % self.accumulation_steps != 0:
            return False
        self.optimizer_step()
        return True

    def optimizer_step(self) -> None:
        if self.loss_sync == "micro":
            acc = self._acc_host
        else:
            acc = float(self._reduce(self._acc_dev).item()) / self.world_size if self._acc_dev is not None else 0.0
        self.loss_list.append(acc)                            # hp:336
        lr = lr_at(self.t, self.initial_lr, self.warmup_steps, self.total_steps, self.schedule)  # hp:338-344
        self.lr_list.append(lr)
        self.t += 1                                           # hp:350
        self.stepper.step(lr, self.t)                         # hp:352-398
        self._acc_host, self._acc_dev = 0.0, None             # hp:400

    def train_epoch(self, dataloader, epoch: int = 0) -> List[float]:
        """hp:316-335 for one epoch: every micro-batch of this rank's shard.  As the reference does at
        each epoch start (hp:317), the accumulated loss restarts at 0: micro-batches of a previous
        epoch that did not complete an accumulation window are not carried into this epoch's log
        (their gradients are, as in the reference: nothing clears .grad between epochs)."""
        sampler = getattr(dataloader, "sampler", None)
        if hasattr(sampler, "set_epoch"):
            sampler.set_epoch(epoch)
        self.micro = 0
        self._acc_host, self._acc_dev = 0.0, None             # hp:317
        for batch in dataloader:
            self.micro_step(batch)
        return self.loss_list
