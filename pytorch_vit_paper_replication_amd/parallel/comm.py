"""Python face of the native RCCL communicator (``csrc/comm.cpp``).

Bootstrap: rank 0 asks RCCL for an ``ncclUniqueId`` and the 128 bytes travel to the other ranks over
the already-initialised ``torch.distributed`` group (``broadcast_object_list``); every rank then
joins the communicator for its own GPU. After that, collectives never touch torch's process group:
they run on the communicator's high-priority HIP stream, event-ordered against the caller's stream.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist

from .. import _ext


class NativeCommunicator:
    def __init__(self, impl, device: torch.device):
        self._c = impl
        self.device = device
        self.rank = impl.rank
        self.world = impl.world

    @classmethod
    def create(cls, device: torch.device, process_group=None) -> "NativeCommunicator":
        ext = _ext.ext()
        if not ext.rccl_available():
            raise RuntimeError("RCCL not loadable: " + ext.rccl_error())
        rank = dist.get_rank(process_group)
        world = dist.get_world_size(process_group)
        obj = [ext.rccl_unique_id() if rank == 0 else None]
        src = dist.get_global_rank(process_group, 0) if process_group is not None else 0
        dist.broadcast_object_list(obj, src=src, group=process_group, device=device)
        idx = device.index if device.index is not None else torch.cuda.current_device()
        return cls(ext.Communicator(obj[0], rank, world, idx), device)

    # all collectives are stream-ordered and asynchronous; wait(h) joins them into the caller's stream
    def all_reduce(self, t: torch.Tensor, average: bool = True, algo: str = "rccl") -> int:
        """``algo="mesh"``: the framework's own schedule (csrc/comm_core.h: reduce-scatter + all-gather
        as grouped point-to-point transfers to every peer at once, fp32); else RCCL's all-reduce."""
        if algo == "mesh":
            return self._c.all_reduce_mesh_async(t, average)
        return self._c.all_reduce_async(t, average)

    def reserve_mesh(self, max_numel: int) -> None:
        """Size the mesh all-reduce's scratch for messages up to ``max_numel`` fp32 (at setup)."""
        self._c.reserve_mesh(int(max_numel))

    def reduce_scatter(self, inp: torch.Tensor, out: torch.Tensor, average: bool = True) -> int:
        return self._c.reduce_scatter_async(inp, out, average)

    def all_gather(self, inp: torch.Tensor, out: torch.Tensor) -> int:
        return self._c.all_gather_async(inp, out)

    def broadcast(self, t: torch.Tensor, root: int = 0) -> int:
        return self._c.broadcast_async(t, root)

    def wait(self, handle: int) -> None:
        self._c.wait(handle)

    def wait_all(self) -> None:
        self._c.wait_all()

    def barrier(self) -> None:
        self._c.barrier()

    def destroy(self) -> None:
        self._c.destroy()


_DEFAULT: Optional[NativeCommunicator] = None


def default_communicator(device: Optional[torch.device] = None) -> NativeCommunicator:
    """Process-wide communicator over the default group (created on first use)."""
    global _DEFAULT
    if _DEFAULT is None:
        dev = device or torch.device("cuda", torch.cuda.current_device())
        _DEFAULT = NativeCommunicator.create(dev)
    return _DEFAULT
