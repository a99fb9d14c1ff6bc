"""Process-group bootstrap: one process per GPU, ``torch.distributed`` over RCCL (backend "nccl" on
ROCm) with the torchrun environment (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT),
or gloo for CPU-only processes (tests)."""
from __future__ import annotations

import datetime
import os
from typing import Optional, Tuple

import torch
import torch.distributed as dist


def env_world() -> Tuple[int, int, int]:
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def is_dist() -> bool:
    return dist.is_available() and dist.is_initialized()


def rank() -> int:
    return dist.get_rank() if is_dist() else 0


def world_size() -> int:
    return dist.get_world_size() if is_dist() else 1


def is_main() -> bool:
    return rank() == 0


# RCCL channel budget while gradients all-reduce under the backward. One RCCL channel is one
# workgroup resident on a CU for the collective's lifetime, and the GEMM / attention kernels it
# overlaps size their grids to the 256 CUs, so every channel steals a CU from them. 16 channels
# (6 % of the CUs) still give two per xGMI link (7 links per MI355X); the ViT-B/16 gradients
# (330 MB fp32 per step at 8 ranks) then need about 2 x 7/8 x 330 MB / (16 x ~20 GB/s) ~ 2 ms per
# step, under a 50-70 ms backward at 512 images per GPU: the collective stays hidden with the
# budget, and the GEMMs keep 94 % of the chip. Override: PVR_RCCL_CHANNELS=N (0 = RCCL's own
# choice) or set NCCL_MAX_NCHANNELS yourself.
RCCL_CHANNELS = 16


def _rccl_budget() -> None:
    if "NCCL_MAX_NCHANNELS" in os.environ:
        return
    n = int(os.environ.get("PVR_RCCL_CHANNELS", str(RCCL_CHANNELS)))
    if n > 0:
        os.environ["NCCL_MAX_NCHANNELS"] = str(n)


def init_distributed(backend: Optional[str] = None, timeout_s: int = 600) -> Tuple[int, int, torch.device]:
    """Initialise the default process group from the environment if WORLD_SIZE > 1.

    Returns (rank, world_size, device). With one process nothing is initialised. On the RCCL
    backend the channel budget above is applied first (RCCL reads it at communicator creation).
    """
    r, w, lr = env_world()
    use_cuda = torch.cuda.is_available() and backend != "gloo"
    device = torch.device("cuda", lr) if use_cuda else torch.device("cpu")
    if use_cuda:
        torch.cuda.set_device(device)
    if w > 1 and not is_dist():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        be = backend or ("nccl" if use_cuda else "gloo")
        kw = dict(backend=be, rank=r, world_size=w, timeout=datetime.timedelta(seconds=timeout_s))
        if be == "nccl":
            kw["device_id"] = device
            _rccl_budget()
        dist.init_process_group(**kw)
    return r, w, device


def barrier():
    if is_dist():
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def destroy():
    if is_dist():
        dist.destroy_process_group()


def all_reduce_max(x: float, device=None) -> float:
    if not is_dist():
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device or ("cuda" if dist.get_backend() == "nccl" else "cpu"))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
