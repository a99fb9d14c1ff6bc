"""Model summary with ``torchinfo.summary``'s accounting (used at MAIN.ipynb:2317-2322, :2653-2660 and
EX.ipynb:17/30/53; torchinfo is not installed on the target image).

The table and the totals follow torchinfo's rules, so the figures printed in the reference notebooks
are reproduced exactly (ViT-B/16, 3 classes, batch 32: 85,800,963 params, 5.52 G mult-adds, input
19.27 MB, forward/backward 3330.74 MB, params 229.20 MB, total 3579.21 MB):

* rows are the modules that ran, in execution order, down to ``depth``; a container that never ran
  itself but holds modules that did (an ``nn.ModuleList``) is shown with ``--`` shapes;
* ``Param #`` is the module's own (non-child) parameter count while its children are displayed, its
  recursive total once ``depth`` hides them (in parentheses when none of them is trainable);
* mult-adds, params size and forward/backward size are sums over executed LEAF modules: a leaf's
  ``weight``/``bias`` contribute ``numel × batch`` (``numel × batch × output pixels`` for convolutions),
  other ``*weight*``/``*bias*`` tensors ``numel × out[0] × out[1]``; the forward/backward size is twice
  the output bytes of executed leaves that own parameters. Attention (``nn.MultiheadAttention`` and
  this package's ``SelfAttention``, which calls its ``out_proj`` functionally just like it) is not a
  leaf, so its projections and the score GEMMs are not in the mult-add count — that is torchinfo's
  figure, not the model's true FLOPs (``bench.py`` prices its MFU on the exact GEMM FLOPs).

On a GPU model the summary forward runs the module-by-module path (``_ext.reference_path``): the
fused encoder would bypass the per-module hooks the accounting needs.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence

import torch
from torch import nn

from .. import _ext

_ALL_COLS = ("input_size", "output_size", "num_params", "params_percent", "kernel_size", "mult_adds",
             "trainable")
_HEADERS = {"input_size": "Input Shape", "output_size": "Output Shape", "num_params": "Param #",
            "params_percent": "Param %", "kernel_size": "Kernel Shape", "mult_adds": "Mult-Adds",
            "trainable": "Trainable"}


def count_params(model: nn.Module, trainable_only: bool = False) -> int:
    return sum(p.numel() for p in model.parameters() if p.requires_grad or not trainable_only)


def _first_tensor(x: Any) -> Optional[torch.Tensor]:
    if torch.is_tensor(x):
        return x
    if isinstance(x, (list, tuple)):
        for e in x:
            t = _first_tensor(e)
            if t is not None:
                return t
    if isinstance(x, dict):
        for e in x.values():
            t = _first_tensor(e)
            if t is not None:
                return t
    return None


@dataclass
class LayerInfo:
    module: nn.Module
    var_name: str
    depth: int
    parent: Optional["LayerInfo"]
    children: List["LayerInfo"] = field(default_factory=list)
    order: Optional[int] = None          # first-execution index (None: never ran)
    input_shape: Optional[List[int]] = None
    output_shape: Optional[List[int]] = None
    output_bytes: int = 0
    macs: int = 0

    @property
    def class_name(self) -> str:
        return type(self.module).__name__

    @property
    def is_leaf(self) -> bool:
        return not any(True for _ in self.module.children())

    @property
    def num_params(self) -> int:
        return sum(p.numel() for p in self.module.parameters())

    @property
    def trainable_params(self) -> int:
        return sum(p.numel() for p in self.module.parameters() if p.requires_grad)

    @property
    def param_bytes(self) -> int:
        return sum(p.numel() * p.element_size() for p in self.module.parameters())

    @property
    def kernel_size(self) -> Optional[List[int]]:
        k = getattr(self.module, "kernel_size", None)
        return list(k) if isinstance(k, (tuple, list)) else ([k] if isinstance(k, int) else None)

    def first_order(self) -> Optional[int]:
        """Execution index of this module or, for a container that never ran, of its first
        descendant that did."""
        if self.order is not None:
            return self.order
        kids = [c.first_order() for c in self.children]
        kids = [k for k in kids if k is not None]
        return min(kids) if kids else None

    def leaf_macs(self) -> int:
        out = self.output_shape
        if not out:
            return 0
        conv = "Conv" in self.class_name
        macs = 0
        for name, p in self.module.named_parameters():
            if name in ("weight", "bias"):
                macs += p.numel() * (math.prod(out[:1] + out[2:]) if conv else out[0])
            elif "weight" in name or "bias" in name:
                macs += p.numel() * math.prod(out[:2])
        return macs


class ModelSummary:
    """Result of :func:`summary`: ``str()`` is the table; the totals are attributes (bytes / counts)."""

    def __init__(self, root: LayerInfo, depth: int, col_names: Sequence[str], col_width: int,
                 input_bytes: int, total_params: int, trainable_params: int):
        self.root = root
        self.depth = depth
        self.col_names = tuple(col_names)
        self.col_width = col_width
        layers = list(_walk(root))
        ran_leaves = [li for li in layers if li.order is not None and li.is_leaf]
        self.total_params = total_params
        self.trainable_params = trainable_params
        self.total_mult_adds = sum(li.macs for li in ran_leaves)
        self.input_bytes = input_bytes
        self.params_bytes = sum(li.param_bytes for li in ran_leaves)
        self.fwd_bwd_bytes = 2 * sum(li.output_bytes for li in ran_leaves if li.num_params > 0)
        self.rows = [li for li in layers if li.depth <= depth and li.first_order() is not None]

    # -- formatting -------------------------------------------------------------------------
    def _params_str(self, li: LayerInfo) -> str:
        n = li.num_params
        if n == 0:
            return "--"
        shown = [c for c in li.children if c.first_order() is not None]
        if li.depth == self.depth or not shown:  # children hidden (depth) or never ran: the total
            s = f"{n:,}"
            return s if li.trainable_params else f"({s})"
        own = n - sum(c.num_params for c in shown)
        return f"{own:,}" if own > 0 else "--"

    def _cell(self, li: LayerInfo, col: str) -> str:
        if col == "input_size":
            return str(li.input_shape) if li.input_shape is not None else "--"
        if col == "output_size":
            return str(li.output_shape) if li.output_shape is not None else "--"
        if col == "num_params":
            return self._params_str(li)
        if col == "params_percent":
            return f"{100.0 * li.num_params / max(1, self.total_params):.2f}%" if li.num_params else "--"
        if col == "kernel_size":
            k = li.kernel_size
            return str(k) if k else "--"
        if col == "mult_adds":
            m = sum(x.macs for x in _walk(li) if x.order is not None and x.is_leaf)
            return f"{m:,}" if m else "--"
        if col == "trainable":
            n, t = li.num_params, li.trainable_params
            return "--" if n == 0 else ("True" if t == n else ("False" if t == 0 else "Partial"))
        raise ValueError(col)

    @staticmethod
    def _prefix(depth: int) -> str:
        if depth == 0:
            return ""
        if depth == 1:
            return "├─"
        return "│    " * (depth - 1) + "└─"

    def __str__(self) -> str:
        names = [self._prefix(li.depth) + f"{li.class_name} ({li.var_name})" for li in self.rows]
        name_w = max([len("Layer (type (var_name))")] + [len(n) for n in names]) + 2
        w = self.col_width
        width = name_w + w * len(self.col_names)
        bar = "=" * width
        head = f"{'Layer (type (var_name))':<{name_w}}" + "".join(f"{_HEADERS[c]:<{w}}" for c in self.col_names)
        lines = [bar, head.rstrip(), bar]
        for n, li in zip(names, self.rows):
            lines.append((f"{n:<{name_w}}" + "".join(f"{self._cell(li, c):<{w}}" for c in self.col_names)).rstrip())
        ma = self.total_mult_adds
        unit, div = ("G", 1e9) if ma >= 1e9 else (("M", 1e6) if ma >= 1e6 else ("K", 1e3))
        lines += [bar,
                  f"Total params: {self.total_params:,}",
                  f"Trainable params: {self.trainable_params:,}",
                  f"Non-trainable params: {self.total_params - self.trainable_params:,}",
                  f"Total mult-adds ({unit}): {ma / div:.2f}",
                  bar,
                  f"Input size (MB): {self.input_mb:.2f}",
                  f"Forward/backward pass size (MB): {self.fwd_bwd_mb:.2f}",
                  f"Params size (MB): {self.params_mb:.2f}",
                  f"Estimated Total Size (MB): {self.total_mb:.2f}",
                  bar]
        return "\n".join(lines)

    __repr__ = __str__

    def __contains__(self, text: str) -> bool:
        return text in str(self)

    # torchinfo rounds each component to MB before adding them up
    @property
    def input_mb(self) -> float:
        return round(self.input_bytes / 1e6, 2)

    @property
    def fwd_bwd_mb(self) -> float:
        return round(self.fwd_bwd_bytes / 1e6, 2)

    @property
    def params_mb(self) -> float:
        return round(self.params_bytes / 1e6, 2)

    @property
    def total_mb(self) -> float:
        return round(self.input_mb + self.fwd_bwd_mb + self.params_mb, 2)

    def to_dict(self) -> Dict[str, Any]:
        return {"total_params": self.total_params, "trainable_params": self.trainable_params,
                "total_mult_adds": self.total_mult_adds, "input_mb": self.input_mb,
                "fwd_bwd_mb": self.fwd_bwd_mb, "params_mb": self.params_mb, "total_mb": self.total_mb}


def _walk(li: LayerInfo):
    yield li
    kids = sorted((c for c in li.children if c.first_order() is not None), key=lambda c: c.first_order())
    for c in kids:
        yield from _walk(c)


def _build_tree(mod: nn.Module, name: str, depth: int, parent: Optional[LayerInfo]) -> LayerInfo:
    li = LayerInfo(module=mod, var_name=name, depth=depth, parent=parent)
    for cname, child in mod.named_children():
        li.children.append(_build_tree(child, cname, depth + 1, li))
    return li


def summary(model: nn.Module, input_size: Optional[Sequence[int]] = None, input_data: Any = None,
            depth: int = 3, col_names: Sequence[str] = ("input_size", "output_size", "num_params", "trainable"),
            col_width: int = 25, device: Any = None, dtype: torch.dtype = torch.float32,
            print_out: bool = True, row_settings: Any = None) -> ModelSummary:
    """torchinfo-compatible summary of ``model`` run on ``input_data`` (or zeros of ``input_size``).

    ``row_settings`` is accepted for call-compatibility with the notebooks (the ``var_names`` layout is
    the only one produced). The model's train/eval mode and requires_grad flags are left untouched.
    """
    for c in col_names:
        if c not in _ALL_COLS:
            raise ValueError(f"unknown column {c!r}; choose from {_ALL_COLS}")
    if device is None:
        p = next(model.parameters(), None)
        device = p.device if p is not None else torch.device("cpu")
    if input_data is None:
        if input_size is None:
            raise ValueError("pass input_size or input_data")
        input_data = torch.zeros(*input_size, device=device, dtype=dtype)
    args = input_data if isinstance(input_data, (list, tuple)) else (input_data,)
    input_bytes = sum(t.numel() * t.element_size() for t in args if torch.is_tensor(t))

    root = _build_tree(model, type(model).__name__, 0, None)
    counter = [0]
    hooks = []

    def make_hook(li: LayerInfo):
        def hook(mod, a, out):
            if li.order is None:
                li.order = counter[0]
                counter[0] += 1
                t_in = _first_tensor(a)  # positional args only: keyword-called modules show "--"
                li.input_shape = list(t_in.shape) if t_in is not None else None
                t_out = _first_tensor(out)
                li.output_shape = list(t_out.shape) if t_out is not None else None
            t_out = _first_tensor(out)
            if t_out is not None:
                li.output_bytes += t_out.numel() * t_out.element_size()
            if li.is_leaf:
                li.macs += li.leaf_macs()
        return hook

    for li in _walk_all(root):
        hooks.append(li.module.register_forward_hook(make_hook(li)))
    modes = [(m, m.training) for m in model.modules()]
    try:
        model.eval()
        with torch.no_grad(), _ext.reference_path():
            model(*args)
    finally:
        for m, t in modes:
            m.training = t
        for h in hooks:
            h.remove()
    res = ModelSummary(root, depth, col_names, col_width, input_bytes, count_params(model),
                       count_params(model, trainable_only=True))
    if print_out:
        print(res)
    return res


def _walk_all(li: LayerInfo):
    yield li
    for c in li.children:
        yield from _walk_all(c)
