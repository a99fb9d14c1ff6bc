"""Checkpointing.

``save_model`` keeps the reference contract (GM/utils.py:7-35): creates the directory, asserts a
``.pth``/``.pt`` suffix, prints ``[INFO] Saving model to: ...`` and writes ``model.state_dict()`` —
here as fp32 CPU tensors with their own storages, so the file loads into the reference ``ViT``
(and vice versa) with plain ``torch.load(..., weights_only=True)`` even though the live parameters
are views into the fused path's flat store.

New: ``load_model`` and full training-state ``save_checkpoint``/``load_checkpoint`` (model,
optimizer, scheduler, epoch, RNG, results, and the fused path's runtime state: the device dropout
counter and the fp8 delayed-scaling histories) for a bit-exact resume — the reference had no load
path at all (GM/utils.py:7-35 only saves).
Only rank 0 writes under torch.distributed.
"""
from __future__ import annotations

import os
from pathlib import Path
from typing import Any, Dict, Optional

import torch


def _rank0() -> bool:
    d = torch.distributed
    return not (d.is_available() and d.is_initialized()) or d.get_rank() == 0


def _unwrap(model):
    return getattr(model, "module", model)


def portable_state_dict(model: torch.nn.Module) -> Dict[str, torch.Tensor]:
    return {k: v.detach().to("cpu", copy=True).contiguous() for k, v in _unwrap(model).state_dict().items()}


def save_model(model: torch.nn.Module, target_dir: str, model_name: str):
    target_dir_path = Path(target_dir)
    target_dir_path.mkdir(parents=True, exist_ok=True)
    assert model_name.endswith(".pth") or model_name.endswith(".pt"), "model_name should end with '.pt' or '.pth'"
    model_save_path = target_dir_path / model_name
    if _rank0():
        print(f"[INFO] Saving model to: {model_save_path}")
        torch.save(obj=portable_state_dict(model), f=model_save_path)
    return model_save_path


def load_model(model: torch.nn.Module, path: str, strict: bool = True, map_location="cpu"):
    sd = torch.load(path, map_location=map_location, weights_only=True)
    return _unwrap(model).load_state_dict(sd, strict=strict)


def save_checkpoint(target_dir: str, model: torch.nn.Module, optimizer=None, lr_scheduler=None, epoch: int = 0,
                    results: Optional[Dict[str, Any]] = None, name: str = "checkpoint.pt") -> Optional[Path]:
    if not _rank0():
        return None
    d = Path(target_dir)
    d.mkdir(parents=True, exist_ok=True)
    state = {
        "model": portable_state_dict(model),
        "epoch": int(epoch),
        "results": results or {},
        "torch_rng": torch.get_rng_state(),
    }
    if torch.cuda.is_available():
        state["cuda_rng"] = [s.cpu() for s in torch.cuda.get_rng_state_all()]
    if optimizer is not None:
        osd = optimizer.state_dict()
        for st in osd.get("state", {}).values():
            for k, v in list(st.items()):
                if torch.is_tensor(v):
                    st[k] = v.detach().to("cpu", copy=True)
        state["optimizer"] = osd
    if lr_scheduler is not None:
        state["lr_scheduler"] = lr_scheduler.state_dict()
    rt = getattr(_unwrap(model), "runtime_state_dict", None)
    if rt is not None:
        # fused-path state outside state_dict(): the device dropout counter and the fp8 scaling
        # histories; without them a resumed run draws other dropout masks / re-calibrates fp8
        state["runtime"] = rt()
    tmp = d / (name + ".tmp")
    torch.save(state, tmp)
    os.replace(tmp, d / name)
    return d / name


def load_checkpoint(path: str, model: torch.nn.Module, optimizer=None, lr_scheduler=None, map_location="cpu",
                    restore_rng: bool = True) -> Dict[str, Any]:
    """Restores state saved by ``save_checkpoint``; returns ``{"epoch", "results"}``.

    The file is read with ``weights_only=True``: everything ``save_checkpoint`` writes (tensors,
    dicts/lists of numbers, the optimizer and LR-scheduler state dicts, RNG byte tensors) loads
    without unpickling arbitrary objects, so a ``--resume`` path cannot execute code."""
    state = torch.load(path, map_location=map_location, weights_only=True)
    _unwrap(model).load_state_dict(state["model"])
    if optimizer is not None and "optimizer" in state:
        optimizer.load_state_dict(state["optimizer"])
    if lr_scheduler is not None and "lr_scheduler" in state:
        lr_scheduler.load_state_dict(state["lr_scheduler"])
    if "runtime" in state and hasattr(_unwrap(model), "load_runtime_state_dict"):
        _unwrap(model).load_runtime_state_dict(state["runtime"])
    if restore_rng and "torch_rng" in state:
        torch.set_rng_state(state["torch_rng"])
        if torch.cuda.is_available() and "cuda_rng" in state:
            try:
                torch.cuda.set_rng_state_all(state["cuda_rng"])
            except Exception:
                pass
    return {"epoch": state.get("epoch", 0), "results": state.get("results", {})}
