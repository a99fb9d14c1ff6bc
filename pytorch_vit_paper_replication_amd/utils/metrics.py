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
