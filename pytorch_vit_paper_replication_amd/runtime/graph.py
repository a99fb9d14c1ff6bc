"""hipGraph capture of a whole training step (forward, loss, backward, clip, Adam).

The fused step is ~150-300 kernel launches plus autograd/Python bookkeeping. For large batches
the GPU hides that host time; for small per-GPU batches (fine-tuning, inference-sized steps) it
does not. ``GraphedTrainStep`` records one step into a ``torch.cuda.CUDAGraph``. On ROCm this is
a hipGraph, the MI355X-native replacement for a tracing compiler. Each
later step is then one ``hipGraphLaunch``, replayed against static input buffers.

What makes the fused step capture-safe:
  * no host synchronisation anywhere in the step (device-side metrics, clip and non-finite checks);
  * ``FusedAdam.graph_mode()``: lr / bias corrections come from a persistent device table that
    ``graph_prepare()`` refreshes before each replay, so LR schedules keep working;
  * dropout seeds advance on the device (``ViT._dropout_seed`` increments a device counter);
  * the weight-gradient side stream forks / joins with events, which capture as graph edges;
  * every scratch tensor is allocated from the graph's private memory pool during capture.
"""
from __future__ import annotations

from typing import Callable, Optional

import torch


class GraphedTrainStep:
    def __init__(self, model: torch.nn.Module, optimizer, loss_fn: Callable, sample_x: torch.Tensor,
                 sample_y: torch.Tensor, clip_norm: Optional[float] = 1.0, warmup: int = 3,
                 scheduler=None):
        if not sample_x.is_cuda:
            raise ValueError("graph capture needs CUDA/HIP tensors")
        self.model, self.optimizer, self.loss_fn = model, optimizer, loss_fn
        self.clip_norm = clip_norm
        self.scheduler = scheduler
        self.static_x = sample_x.clone()
        self.static_y = sample_y.clone()
        # eager warm-up on a side stream (lazy allocations, store / transposed-weight setup, fp8
        # calibration) as required before capture
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(max(1, warmup)):
                self._body()
                if self.scheduler is not None:
                    self.scheduler.step()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        optimizer.graph_mode(True)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.static_loss = self._body()
        torch.cuda.synchronize()

    def _body(self) -> torch.Tensor:
        self.model.train()
        loss = self.loss_fn(self.model(self.static_x), self.static_y)
        self.optimizer.zero_grad()
        from ..ops.fused_vit import backward

        backward(loss)
        self.optimizer.step(clip_norm=self.clip_norm)
        return loss.detach()

    def __call__(self, x: Optional[torch.Tensor] = None, y: Optional[torch.Tensor] = None) -> torch.Tensor:
        """One training step on (x, y) (copied into the static buffers); returns the device loss."""
        if x is not None:
            self.static_x.copy_(x, non_blocking=True)
        if y is not None:
            self.static_y.copy_(y, non_blocking=True)
        self.optimizer.graph_prepare()
        self.graph.replay()
        if self.scheduler is not None:
            self.scheduler.step()
        return self.static_loss
