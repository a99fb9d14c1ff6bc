"""Model introspection (stand-in for ``torchinfo.summary`` used at MAIN.ipynb:2317-2322, :2653-2660;
torchinfo is not installed on the target image): per-module output shapes and parameter counts."""
from __future__ import annotations

from typing import List, Sequence, Tuple

import torch
from torch import nn


def count_params(model: nn.Module, trainable_only: bool = False) -> int:
    return sum(p.numel() for p in model.parameters() if p.requires_grad or not trainable_only)


def summary(model: nn.Module, input_size: Sequence[int], depth: int = 2, device="cpu", print_out: bool = True) -> str:
    rows: List[Tuple[str, str, str, int, bool]] = []
    hooks = []

    def reg(name, mod, d):
        def hook(m, inp, out):
            i = inp[0] if isinstance(inp, (tuple, list)) and inp else inp
            o = out[0] if isinstance(out, (tuple, list)) else out
            n_own = sum(p.numel() for p in m.parameters(recurse=False))
            n_all = sum(p.numel() for p in m.parameters())
            tr = all(p.requires_grad for p in m.parameters()) if n_all else True
            rows.append(("  " * d + f"{name} ({type(m).__name__})",
                         str(list(i.shape)) if torch.is_tensor(i) else "-",
                         str(list(o.shape)) if torch.is_tensor(o) else "-", n_all if d == depth or not list(m.children()) else n_own, tr))
        hooks.append(mod.register_forward_hook(hook))

    def walk(mod, prefix, d):
        for name, child in mod.named_children():
            full = f"{prefix}.{name}" if prefix else name
            reg(full, child, d)
            if d < depth:
                walk(child, full, d + 1)

    walk(model, "", 0)
    was = model.training
    model.eval()
    with torch.no_grad():
        model(torch.zeros(*input_size, device=device))
    model.train(was)
    for h in hooks:
        h.remove()
    total = count_params(model)
    trainable = count_params(model, True)
    lines = [f"{'Layer (type)':60s} {'Input Shape':22s} {'Output Shape':22s} {'Param #':>12s}", "=" * 120]
    for name, i, o, n, _ in rows:
        lines.append(f"{name[:60]:60s} {i:22s} {o:22s} {n:12,d}")
    lines += ["=" * 120, f"Total params: {total:,}", f"Trainable params: {trainable:,}",
              f"Non-trainable params: {total - trainable:,}",
              f"Params size (MB): {total * 4 / 1e6:.2f}"]
    s = "\n".join(lines)
    if print_out:
        print(s)
    return s
