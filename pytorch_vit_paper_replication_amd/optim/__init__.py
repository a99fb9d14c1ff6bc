"""Optimizers and schedules (reference recipe: MAIN.ipynb:2792-2960)."""
from .adam import FusedAdam
from .schedule import param_groups_weight_decay, warmup_decay_steps, warmup_linear_decay

__all__ = ["FusedAdam", "param_groups_weight_decay", "warmup_decay_steps", "warmup_linear_decay"]
