"""Profiling hooks: ROCTX ranges (visible in rocprofv3 --marker-trace) and a torch.profiler wrapper
that writes a per-kernel summary table (proves which HIP kernels run on the hot path)."""
from __future__ import annotations

import contextlib
import ctypes
import os
from typing import Optional

import torch

_ROCTX = None


def _roctx():
    global _ROCTX
    if _ROCTX is None:
        _ROCTX = False
        for name in ("libroctx64.so", "/opt/rocm/lib/libroctx64.so"):
            try:
                lib = ctypes.CDLL(name)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                _ROCTX = lib
                break
            except OSError:
                continue
    return _ROCTX or None


@contextlib.contextmanager
def range_push(name: str):
    lib = _roctx() if os.environ.get("PVR_ROCTX", "0") == "1" else None
    if lib is not None:
        lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        if lib is not None:
            lib.roctxRangePop()


def profile_steps(fn, steps: int = 3, out_path: Optional[str] = None, row_limit: int = 40) -> str:
    acts = [torch.profiler.ProfilerActivity.CPU]
    if torch.cuda.is_available():
        acts.append(torch.profiler.ProfilerActivity.CUDA)
    with torch.profiler.profile(activities=acts) as prof:
        for _ in range(steps):
            fn()
        if torch.cuda.is_available():
            torch.cuda.synchronize()
    key = "cuda_time_total" if torch.cuda.is_available() else "cpu_time_total"
    table = prof.key_averages().table(sort_by=key, row_limit=row_limit)
    if out_path:
        with open(out_path, "w") as f:
            f.write(table)
    return table
