"""Data parallelism: RCCL-over-xGMI bucketed gradient all-reduce (ddp) and process-group helpers."""
from .ddp import DistributedDataParallel
from .dist import barrier, destroy, init_distributed, is_dist, is_main, rank, world_size

__all__ = ["DistributedDataParallel", "init_distributed", "barrier", "destroy", "is_dist", "is_main", "rank",
           "world_size"]
