"""Training / evaluation engine with the reference API (GM/engine.py:9-211).

``train(model, train_dataloader, test_dataloader, optimizer, loss_fn, lr_scheduler, epochs, device)``
returns ``{"train_loss": [...], "train_acc": [...], "test_loss": [...], "test_acc": [...]}`` and prints
``Epoch: n | train_loss: .. | train_acc: .. | test_loss: .. | test_acc: ..`` per epoch, exactly like
the reference. Preserved semantics:
  * the scheduler steps once per batch, gradients are clipped to global norm 1.0 before the step;
  * metrics are the mean over batches of per-batch means (a partial last batch weighs like a full one);
  * the train accuracy uses argmax(softmax(logits)) (== argmax(logits)), test uses argmax(logits).

MI355X-oriented differences (no behaviour change):
  * per-batch loss/accuracy accumulate on the device; the host syncs once per epoch instead of
    twice per batch (the reference's ``.item()`` calls, GM/engine.py:54,74,121,125);
  * with :class:`~..optim.FusedAdam` the clip runs inside the optimizer (device-side coefficient,
    no sync) and ``nn.CrossEntropyLoss()`` is executed by the fused softmax-xent kernel, whose
    per-row argmax == label flags also give the accuracy (no separate argmax / eq / sum);
  * under ``torch.distributed`` metrics are all-reduced across ranks and only rank 0 prints;
  * on a GPU the next batch's host->device copy runs on a copy stream while the current step
    computes (:class:`~.data.prefetch.DevicePrefetcher`, K17) instead of a blocking ``.to(device)``.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import torch
from torch import nn

try:
    from tqdm.auto import tqdm
except Exception:  # pragma: no cover
    def tqdm(x, **_):
        return x

from .data.prefetch import prefetch
from .ops import fused_vit
from .ops.fused_vit import cross_entropy
from .utils.profiling import range_push


def _is_dist() -> bool:
    return torch.distributed.is_available() and torch.distributed.is_initialized()


def _rank0() -> bool:
    return not _is_dist() or torch.distributed.get_rank() == 0


def _fused_loss(loss_fn):
    """Use the fused kernel for a default nn.CrossEntropyLoss (same math and reduction)."""
    if isinstance(loss_fn, nn.CrossEntropyLoss) and loss_fn.weight is None and loss_fn.reduction == "mean" \
            and loss_fn.label_smoothing == 0.0 and loss_fn.ignore_index == -100:
        return cross_entropy
    return loss_fn


def _accumulate(sums: torch.Tensor, loss: torch.Tensor, logits: torch.Tensor, y: torch.Tensor, lf) -> None:
    """sums += [batch loss, batch accuracy] on the device. With the fused cross-entropy the kernel's
    per-row argmax == label flags are summed by one small HIP kernel; otherwise argmax / eq / sum."""
    with torch.no_grad():
        corr = fused_vit.last_correct if lf is cross_entropy else None
        if corr is not None and sums.is_cuda and corr.numel() == logits.shape[0]:
            from . import _ext

            _ext.ext().metrics_accum(sums, loss.detach().float().reshape(1), corr)
            return
        acc = (logits.argmax(dim=1) == y).sum().float() / logits.shape[0]
        sums += torch.stack([loss.detach().float(), acc])


def _clip_and_step(model, optimizer, max_norm: Optional[float]) -> Optional[torch.Tensor]:
    """Clip + optimizer step; returns the pre-clip global gradient norm (a device tensor) or None."""
    from .optim.adam import FusedAdam

    if isinstance(optimizer, FusedAdam):
        optimizer.step(clip_norm=max_norm)
        return optimizer.last_grad_norm
    norm = None
    if max_norm is not None:
        norm = torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=max_norm)
    optimizer.step()
    return norm


def _reduce_means(sums: torch.Tensor, count: int, device) -> Tuple[float, ...]:
    """sums: per-metric sums of per-batch means; returns global mean-of-batch-means."""
    vals = torch.cat([sums.double().reshape(-1), torch.tensor([float(count)], dtype=torch.float64, device=sums.device)])
    if _is_dist():
        if vals.device.type == "cpu" and torch.distributed.get_backend() == "nccl":
            vals = vals.to(device)
        torch.distributed.all_reduce(vals)
    vals = vals.cpu()
    n = max(vals[-1].item(), 1.0)
    return tuple((vals[:-1] / n).tolist())


def _set_sampler_epoch(dataloader, epoch: Optional[int]) -> None:
    """Reshuffle a DistributedSampler per epoch (otherwise every epoch repeats one permutation)."""
    sampler = getattr(dataloader, "sampler", None)
    if epoch is not None and hasattr(sampler, "set_epoch"):
        sampler.set_epoch(epoch)


def train_step(model: torch.nn.Module, dataloader, loss_fn: torch.nn.Module, optimizer: torch.optim.Optimizer,
               lr_scheduler, device, *, max_grad_norm: Optional[float] = 1.0,
               epoch: Optional[int] = None, step_logger=None) -> Tuple[float, float]:
    """One training epoch (reference GM/engine.py:9-79). Returns (train_loss, train_acc).

    ``epoch`` (optional) seeds a ``DistributedSampler``'s shuffle for this epoch. ``step_logger``
    (optional :class:`~.utils.metrics.StepLogger`) gets one record per batch: step time, img/s, lr,
    loss, gradient norm and, under this package's DDP built with ``timing=True``, per-bucket
    all-reduce times — without a host synchronisation per step."""
    _set_sampler_epoch(dataloader, epoch)
    model.train()
    lf = _fused_loss(loss_fn)
    sums = torch.zeros(2, dtype=torch.float32, device=device)
    nb = 0
    for X, y in prefetch(dataloader, device):
        if step_logger is not None:
            step_logger.begin()
        X, y = X.to(device, non_blocking=True), y.to(device, non_blocking=True)
        with range_push("forward"):  # ROCTX ranges (PVR_ROCTX=1, rocprofv3 --marker-trace)
            y_pred = model(X)
            loss = lf(y_pred, y)
        optimizer.zero_grad()
        with range_push("backward"):
            fused_vit.backward(loss)
        with range_push("optimizer"):
            norm = _clip_and_step(model, optimizer, max_grad_norm)
        lr = optimizer.param_groups[0]["lr"]
        lr_scheduler.step()
        _accumulate(sums, loss, y_pred, y, lf)
        if step_logger is not None:
            step_logger.end(batch=X.shape[0], loss=loss, grad_norm=norm, lr=lr, epoch=epoch,
                            ddp=model if hasattr(model, "pop_timing") else None)
        nb += 1
    loss_m, acc_m = _reduce_means(sums, nb, device)
    return loss_m, acc_m


def test_step(model: torch.nn.Module, dataloader, loss_fn: torch.nn.Module, device) -> Tuple[float, float]:
    """One evaluation epoch (reference GM/engine.py:81-130). Returns (test_loss, test_acc)."""
    model.eval()
    lf = _fused_loss(loss_fn)
    sums = torch.zeros(2, dtype=torch.float32, device=device)
    nb = 0
    with torch.inference_mode():
        for X, y in prefetch(dataloader, device):
            X, y = X.to(device, non_blocking=True), y.to(device, non_blocking=True)
            logits = model(X)
            loss = lf(logits, y)
            _accumulate(sums, loss, logits, y, lf)
            nb += 1
    loss_m, acc_m = _reduce_means(sums, nb, device)
    return loss_m, acc_m


def train(model: torch.nn.Module, train_dataloader, test_dataloader, optimizer: torch.optim.Optimizer,
          loss_fn: torch.nn.Module, lr_scheduler, epochs: int, device, *, max_grad_norm: Optional[float] = 1.0,
          checkpoint_dir: Optional[str] = None, metrics_path: Optional[str] = None, start_epoch: int = 0,
          results: Optional[Dict[str, List]] = None, step_metrics_path: Optional[str] = None,
          log_every: int = 50) -> Dict[str, List]:
    """Train and test for ``epochs`` epochs (reference GM/engine.py:132-211).

    ``metrics_path``: one JSONL record per epoch. ``step_metrics_path``: one JSONL record per training
    step (:class:`~.utils.metrics.StepLogger`, flushed every ``log_every`` steps; rank 0 writes).

    Resume (new, optional): ``start_epoch`` epochs are already done (``load_checkpoint(...)["epoch"]``)
    and ``results`` holds their metrics; only epochs ``start_epoch + 1 .. epochs`` run, numbered as
    in the uninterrupted run, and their metrics are appended to ``results``."""
    base = {"train_loss": [], "train_acc": [], "test_loss": [], "test_acc": []}
    results = {k: list((results or {}).get(k, [])) for k in base}
    model.to(device)
    epochs_left = range(start_epoch, epochs)
    it = tqdm(epochs_left) if _rank0() else epochs_left
    step_logger = None
    if step_metrics_path:
        from .utils.metrics import StepLogger

        world = torch.distributed.get_world_size() if _is_dist() else 1
        rank = torch.distributed.get_rank() if _is_dist() else 0
        step_logger = StepLogger(step_metrics_path, flush_every=log_every, rank=rank, world=world,
                                 device=torch.device(device))
    for epoch in it:
        train_loss, train_acc = train_step(model=model, dataloader=train_dataloader, loss_fn=loss_fn,
                                           optimizer=optimizer, lr_scheduler=lr_scheduler, device=device,
                                           max_grad_norm=max_grad_norm, epoch=epoch, step_logger=step_logger)
        if step_logger is not None:
            step_logger.flush()
        test_loss, test_acc = test_step(model=model, dataloader=test_dataloader, loss_fn=loss_fn, device=device)
        if _rank0():
            print(f"Epoch: {epoch + 1} | "
                  f"train_loss: {train_loss:.4f} | "
                  f"train_acc: {train_acc:.4f} | "
                  f"test_loss: {test_loss:.4f} | "
                  f"test_acc: {test_acc:.4f}")
        results["train_loss"].append(train_loss)
        results["train_acc"].append(train_acc)
        results["test_loss"].append(test_loss)
        results["test_acc"].append(test_acc)
        if metrics_path and _rank0():
            from .utils.metrics import append_jsonl

            append_jsonl(metrics_path, {"epoch": epoch + 1, "train_loss": train_loss, "train_acc": train_acc,
                                        "test_loss": test_loss, "test_acc": test_acc})
        if checkpoint_dir:
            from .utils.checkpoint import save_checkpoint

            save_checkpoint(checkpoint_dir, model=model, optimizer=optimizer, lr_scheduler=lr_scheduler,
                            epoch=epoch + 1, results=results)
    return results
