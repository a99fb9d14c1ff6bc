"""Synthetic ImageNet-shaped data generated on the device (benchmarks, smoke tests).

``SyntheticImageNet`` is a map-style dataset (CPU tensors, deterministic per index) usable with any
DataLoader; ``DeviceSyntheticLoader`` is a DataLoader-like iterable that yields batches already on
the device with no host->device traffic — the input pipeline of the images/sec benchmark
(BASELINE.json: "synthetic ImageNet-shaped data with random-init weights").
"""
from __future__ import annotations

from typing import Iterator, Optional, Tuple

import torch
from torch.utils.data import Dataset


class SyntheticImageNet(Dataset):
    def __init__(self, length: int = 1024, image_size: int = 224, num_classes: int = 1000, channels: int = 3,
                 seed: int = 0):
        self.length, self.image_size, self.num_classes, self.channels, self.seed = (
            length, image_size, num_classes, channels, seed)
        self.classes = [f"class_{i}" for i in range(num_classes)]

    def __len__(self):
        return self.length

    def __getitem__(self, i):
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + i)
        x = torch.rand(self.channels, self.image_size, self.image_size, generator=g)
        y = int(torch.randint(0, self.num_classes, (1,), generator=g))
        return x, y


class DeviceSyntheticLoader:
    """Yields ``steps`` batches of ``[B,3,S,S]`` float32 in [0,1) and int64 labels on ``device``.

    With ``fixed=True`` (the default) one batch is generated once and re-yielded, so the timed region
    measures the model step only (the reference's DataLoader cost is not part of the metric).
    """

    def __init__(self, batch_size: int, steps: int, image_size: int = 224, num_classes: int = 1000,
                 device: Optional[torch.device] = None, fixed: bool = True, seed: int = 0, dtype=torch.float32):
        self.batch_size, self.steps, self.image_size, self.num_classes = batch_size, steps, image_size, num_classes
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.fixed, self.seed, self.dtype = fixed, seed, dtype
        self._batch: Optional[Tuple[torch.Tensor, torch.Tensor]] = None
        self.dataset = SyntheticImageNet(steps * batch_size, image_size, num_classes, seed=seed)

    def _make(self, k: int):
        g = torch.Generator(device=self.device).manual_seed(self.seed + k)
        x = torch.rand(self.batch_size, 3, self.image_size, self.image_size, generator=g, device=self.device,
                       dtype=self.dtype)
        y = torch.randint(0, self.num_classes, (self.batch_size,), generator=g, device=self.device)
        return x, y

    def __len__(self):
        return self.steps

    def __iter__(self) -> Iterator[Tuple[torch.Tensor, torch.Tensor]]:
        for k in range(self.steps):
            if self.fixed:
                if self._batch is None:
                    self._batch = self._make(0)
                yield self._batch
            else:
                yield self._make(k)
