"""Copy-stream batch prefetcher (host→device input transfer).

The reference moves every batch with a blocking ``X.to(device)`` at the top of the step
(GM/engine.py:38-39, 105-106), so the H2D copy of batch i+1 never overlaps the compute of batch i.
:class:`DevicePrefetcher` wraps any iterable of ``(X, y, ...)`` tuples and keeps ONE batch in flight:

* the destination tensors are allocated on the consumer (compute) stream, so the caching allocator
  ties them to that stream and no ``record_stream`` is needed (cross-stream ``record_stream`` defers
  frees and was measured to stall the allocator at large batch, see runtime/param_store.py);
* the copy itself runs on a dedicated HIP stream of the default priority (0, the lowest torch
  offers; ``bench.py`` runs the step on a priority -1 stream above it), after an event that orders it
  behind the allocation. A host-to-device copy is executed by a DMA (SDMA) engine, not a compute
  queue, so it does not take compute-queue slots from the step (the process has
  ``GPU_MAX_HW_QUEUES`` = 4 hardware compute queues, which the compute streams share);
* the consumer stream waits on the copy's event right before the batch is handed out — no host
  synchronisation anywhere.

Host tensors should come pinned (``DataLoader(pin_memory=True)``, which ``create_dataloaders`` sets);
unpinned ones are pinned here so the copy stays asynchronous. On a CPU device the wrapper degrades to
``.to(device)``. ``sampler`` / ``dataset`` / ``len()`` pass through, so ``DistributedSampler.set_epoch``
and the engine's batch counting keep working.
"""
from __future__ import annotations

from typing import Any, Iterable, Iterator, Optional

import torch


def _to_device(obj: Any, device: torch.device, copy_stream, alloc_stream) -> Any:
    if isinstance(obj, torch.Tensor):
        if obj.device == device:
            return obj
        if device.type != "cuda":
            return obj.to(device)
        src = obj
        if device.type == "cuda" and src.device.type == "cpu" and not src.is_pinned():
            src = src.pin_memory()
        with torch.cuda.stream(alloc_stream):
            dst = torch.empty(src.shape, dtype=src.dtype, device=device)
        with torch.cuda.stream(copy_stream):
            dst.copy_(src, non_blocking=True)
        return dst
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to_device(o, device, copy_stream, alloc_stream) for o in obj)
    return obj


class DevicePrefetcher:
    """Iterate ``loader`` with the next batch's host→device copy overlapping the current step."""

    def __init__(self, loader: Iterable, device, *, depth: int = 1):
        self.loader = loader
        self.device = torch.device(device)
        if self.device.type == "cuda" and self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.depth = max(1, int(depth))
        self._copy_stream = None

    # pass-throughs the engine and DistributedSampler users rely on
    @property
    def sampler(self):
        return getattr(self.loader, "sampler", None)

    @property
    def dataset(self):
        return getattr(self.loader, "dataset", None)

    def __len__(self) -> int:
        return len(self.loader)  # type: ignore[arg-type]

    def _stream(self):
        if self._copy_stream is None:
            self._copy_stream = torch.cuda.Stream(device=self.device, priority=0)
        return self._copy_stream

    def __iter__(self) -> Iterator:
        if self.device.type != "cuda":
            for batch in self.loader:
                yield _to_device(batch, self.device, None, None)
            return
        cs = self._stream()
        main = torch.cuda.current_stream(self.device)
        pending = []  # [(batch on device, copy-done event)]
        it = iter(self.loader)

        def issue() -> bool:
            try:
                host = next(it)
            except StopIteration:
                return False
            ready = torch.cuda.Event()
            ready.record(main)  # the destination memory is free in the consumer's stream order
            cs.wait_event(ready)
            dev = _to_device(host, self.device, cs, main)
            done = torch.cuda.Event()
            done.record(cs)
            pending.append((dev, done))
            return True

        for _ in range(self.depth):
            if not issue():
                break
        while pending:
            batch, done = pending.pop(0)
            main.wait_event(done)
            issue()  # the next copy runs while the caller computes on `batch`
            yield batch


def prefetch(loader: Iterable, device, enabled: Optional[bool] = None):
    """``DevicePrefetcher(loader, device)`` on a GPU device (or when ``enabled``), else ``loader``."""
    dev = torch.device(device)
    if enabled is None:
        enabled = dev.type == "cuda"
    if not enabled or isinstance(loader, DevicePrefetcher):
        return loader
    return DevicePrefetcher(loader, dev)
