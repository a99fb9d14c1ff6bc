"""Lightweight observability: JSONL metric records and device-synchronised step timers."""
from __future__ import annotations

import json
import time
from typing import Any, Dict, List, Optional

import torch


def append_jsonl(path: str, record: Dict[str, Any]) -> None:
    with open(path, "a") as f:
        f.write(json.dumps(record) + "\n")


class StepTimer:
    """Times GPU work with HIP events (no host sync inside the measured loop)."""

    def __init__(self, enabled: bool = True):
        self.enabled = enabled and torch.cuda.is_available()
        self.events: List = []

    def mark(self):
        if self.enabled:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self.events.append(e)

    def intervals_ms(self) -> List[float]:
        if not self.enabled or len(self.events) < 2:
            return []
        self.events[-1].synchronize()
        return [a.elapsed_time(b) for a, b in zip(self.events[:-1], self.events[1:])]


class WallTimer:
    def __init__(self, sync: bool = True):
        self.sync = sync and torch.cuda.is_available()
        self.t0: Optional[float] = None

    def __enter__(self):
        if self.sync:
            torch.cuda.synchronize()
        self.t0 = time.perf_counter()
        return self

    def __exit__(self, *exc):
        if self.sync:
            torch.cuda.synchronize()
        self.elapsed = time.perf_counter() - self.t0


class StepLogger:
    """Per-step JSONL metrics without a host synchronisation per step (SURVEY.md §5 metrics row).

    ``begin()`` / ``end(...)`` bracket one training step. On a GPU the step time comes from HIP events
    recorded on the current stream, the loss and gradient norm stay device tensors, and a DDP wrapper
    built with ``timing=True`` hands over its per-bucket all-reduce events; everything is resolved
    every ``flush_every`` steps (one sync per flush) and on :meth:`close`. One record per step::

        {"kind": "step", "step": 12, "epoch": 0, "ms": 34.1, "img_s": 7507.3, "lr": 0.00093,
         "loss": 6.91, "grad_norm": 1.84, "batch": 256, "world": 1, "rank": 0,
         "allreduce": [{"bucket": 0, "bytes": 28901376, "ms": 0.41}, ...], "allreduce_ms": 3.2}

    ``ms`` is the device time from the step's first to its last queued kernel (host time on CPU);
    ``img_s`` = ``batch * world / ms``; an all-reduce entry's ``ms`` runs from the moment its bucket
    was ready on the compute stream to the collective's completion (it includes queueing behind the
    previous bucket). Only the rank given ``enabled=True`` writes (default: rank 0).
    """

    SCHEMA = ("kind", "step", "epoch", "ms", "img_s", "lr", "loss", "grad_norm", "batch", "world", "rank",
              "allreduce", "allreduce_ms")

    def __init__(self, path: str, flush_every: int = 50, rank: int = 0, world: int = 1,
                 enabled: Optional[bool] = None, device: Optional[torch.device] = None):
        self.path = path
        self.flush_every = max(1, int(flush_every))
        self.rank, self.world = rank, world
        self.enabled = (rank == 0) if enabled is None else enabled
        dev = device if device is not None else (torch.device("cuda", torch.cuda.current_device())
                                                 if torch.cuda.is_available() else torch.device("cpu"))
        self.cuda = dev.type == "cuda"
        self.step = 0
        self._pending: List[Dict[str, Any]] = []
        self._t0: Any = None

    def begin(self) -> None:
        if not self.enabled:
            return
        if self.cuda:
            self._t0 = torch.cuda.Event(enable_timing=True)
            self._t0.record()
        else:
            self._t0 = time.perf_counter()

    def end(self, batch: int, loss: Optional[torch.Tensor] = None, grad_norm: Optional[torch.Tensor] = None,
            lr: Optional[float] = None, epoch: Optional[int] = None, ddp: Any = None) -> None:
        timing = ddp.pop_timing() if ddp is not None and hasattr(ddp, "pop_timing") else []
        if not self.enabled:
            return
        if self.cuda:
            t1: Any = torch.cuda.Event(enable_timing=True)
            t1.record()
        else:
            t1 = time.perf_counter()
        snap = lambda t: None if t is None else t.detach().reshape(-1)[:1].float().clone()  # noqa: E731
        self._pending.append({"step": self.step, "epoch": epoch, "t0": self._t0, "t1": t1, "batch": batch,
                              "lr": lr, "loss": snap(loss), "grad_norm": snap(grad_norm), "comm": timing})
        self.step += 1
        if len(self._pending) >= self.flush_every:
            self.flush()

    @staticmethod
    def _elapsed_ms(a: Any, b: Any) -> float:
        if isinstance(a, float):
            return (b - a) * 1000.0
        return float(a.elapsed_time(b))

    def flush(self) -> None:
        if not self.enabled or not self._pending:
            return
        if self.cuda:
            # every pending event must have completed before elapsed_time: the DDP per-bucket end
            # events live on the all-reduce timing stream, which the compute stream's last event does
            # not order ("device not ready" otherwise); one device sync per flush
            torch.cuda.synchronize()
        with open(self.path, "a") as f:
            for r in self._pending:
                ms = self._elapsed_ms(r["t0"], r["t1"])
                ar = [{"bucket": i, "bytes": int(nbytes), "ms": round(self._elapsed_ms(s, e), 4)}
                      for i, (nbytes, s, e) in enumerate(r["comm"])]
                rec = {"kind": "step", "step": r["step"], "epoch": r["epoch"], "ms": round(ms, 4),
                       "img_s": round(r["batch"] * self.world / (ms / 1000.0), 2) if ms > 0 else None,
                       "lr": r["lr"], "loss": None if r["loss"] is None else float(r["loss"].item()),
                       "grad_norm": None if r["grad_norm"] is None else float(r["grad_norm"].item()),
                       "batch": r["batch"], "world": self.world, "rank": self.rank, "allreduce": ar,
                       "allreduce_ms": round(sum(a["ms"] for a in ar), 4) if ar else None}
                f.write(json.dumps(rec) + "\n")
        self._pending = []

    def close(self) -> None:
        self.flush()
