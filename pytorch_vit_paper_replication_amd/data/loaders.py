"""``create_dataloaders`` (reference GM/data_setup.py:12-65) plus data-parallel sharding.

Same positional signature and return value ``(train_dataloader, test_dataloader, class_names)``;
train shuffles, test does not, ``pin_memory=True``. Differences, all opt-in or behaviour-neutral:
workers are persistent across epochs (the reference re-spawned ``os.cpu_count()`` processes every
epoch, which dominated its wall clock), and under ``torch.distributed`` each rank
gets a ``DistributedSampler`` shard.
"""
from __future__ import annotations

import os
from typing import Callable, Optional

import torch
from torch.utils.data import DataLoader, DistributedSampler

from .image_folder import ImageFolder
from .synthetic import SyntheticImageNet

NUM_WORKERS = os.cpu_count()


def _dist():
    return torch.distributed.is_available() and torch.distributed.is_initialized()


def _make_loader(ds, batch_size, shuffle, num_workers, pin_memory, distributed, drop_last=False):
    sampler = None
    if distributed:
        sampler = DistributedSampler(ds, shuffle=shuffle, drop_last=drop_last)
        shuffle = False
    kw = {}
    if num_workers and num_workers > 0:
        kw["persistent_workers"] = True
        kw["prefetch_factor"] = 4
    return DataLoader(ds, batch_size=batch_size, shuffle=shuffle, sampler=sampler, num_workers=num_workers or 0,
                      pin_memory=pin_memory and torch.cuda.is_available(), drop_last=drop_last, **kw)


def create_dataloaders(train_dir: str, test_dir: str, transform: Callable, batch_size: int,
                       num_workers: int = NUM_WORKERS, *, pin_memory: bool = True, distributed: Optional[bool] = None,
                       test_transform: Optional[Callable] = None):
    """Returns ``(train_dataloader, test_dataloader, class_names)``."""
    train_data = ImageFolder(train_dir, transform=transform)
    test_data = ImageFolder(test_dir, transform=test_transform or transform)
    class_names = train_data.classes
    dist = _dist() if distributed is None else distributed
    train_dataloader = _make_loader(train_data, batch_size, True, num_workers, pin_memory, dist)
    test_dataloader = _make_loader(test_data, batch_size, False, num_workers, pin_memory, dist)
    return train_dataloader, test_dataloader, class_names


def create_synthetic_dataloaders(batch_size: int, train_len: int = 256, test_len: int = 64, image_size: int = 224,
                                 num_classes: int = 1000, num_workers: int = 0, distributed: Optional[bool] = None):
    """Synthetic stand-in with the same return contract (no dataset download possible offline)."""
    tr = SyntheticImageNet(train_len, image_size, num_classes, seed=1)
    te = SyntheticImageNet(test_len, image_size, num_classes, seed=2)
    dist = _dist() if distributed is None else distributed
    return (_make_loader(tr, batch_size, True, num_workers, False, dist),
            _make_loader(te, batch_size, False, num_workers, False, dist), tr.classes)
