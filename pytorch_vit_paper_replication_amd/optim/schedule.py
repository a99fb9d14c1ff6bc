"""Learning-rate schedules and parameter grouping of the reference recipe.

* ``param_groups_weight_decay`` — MAIN.ipynb:2792-2802: trainable params with ``ndim == 1`` or a
  name ending in ``.bias`` get no weight decay, everything else (incl. class token, position
  embedding, conv and in_proj weights) gets ``weight_decay``.
* ``warmup_linear_decay`` — MAIN.ipynb:2896-2960: ``SequentialLR([LinearLR(1e-6 -> 1, warmup),
  LinearLR(1 -> 0, decay)], milestones=[warmup])`` with ``warmup = int(0.05 * total_steps)``,
  stepped once per batch by the engine. Returns the same torch scheduler objects.
"""
from __future__ import annotations

from typing import Dict, List, Tuple

import torch


def param_groups_weight_decay(model: torch.nn.Module, weight_decay: float = 0.03) -> List[Dict]:
    decay, no_decay = [], []
    for name, param in model.named_parameters():
        if not param.requires_grad:
            continue
        if param.ndim == 1 or name.endswith(".bias"):
            no_decay.append(param)
        else:
            decay.append(param)
    return [{"params": decay, "weight_decay": weight_decay}, {"params": no_decay, "weight_decay": 0.0}]


def warmup_decay_steps(epochs: int, steps_per_epoch: int, warmup_frac: float = 0.05) -> Tuple[int, int, int]:
    total = epochs * steps_per_epoch
    warmup = int(warmup_frac * total)
    return total, warmup, total - warmup


def warmup_linear_decay(optimizer: torch.optim.Optimizer, total_steps: int, warmup_frac: float = 0.05,
                        start_factor: float = 1e-6) -> torch.optim.lr_scheduler.LRScheduler:
    warmup = int(warmup_frac * total_steps)
    decay = total_steps - warmup
    if warmup <= 0:
        return torch.optim.lr_scheduler.LinearLR(optimizer, start_factor=1.0, end_factor=0.0, total_iters=max(decay, 1))
    w = torch.optim.lr_scheduler.LinearLR(optimizer, start_factor=start_factor, end_factor=1.0, total_iters=warmup)
    d = torch.optim.lr_scheduler.LinearLR(optimizer, start_factor=1.0, end_factor=0.0, total_iters=max(decay, 1))
    return torch.optim.lr_scheduler.SequentialLR(optimizer, schedulers=[w, d], milestones=[warmup])
