"""FusedAdam: torch.optim.Adam semantics, one HIP pass over the flat parameter store.

Drop-in for the reference recipe (MAIN.ipynb:2818-2824: two param groups, wd 0.03 / 0.0, coupled L2
weight decay, betas (0.9, 0.999), eps 1e-8) and for AdamW (``decoupled_weight_decay=True``).

On the fused GPU path all parameters live in one ``ParamStore``; a step is
  [optional] global-norm clip:  two deterministic reduction kernels -> {norm, coef, nonfinite} on device
  Adam:                          one kernel: g*coef (+wd*p) -> m, v -> p -> bf16 shadow (and the
                                 transposed bf16 shadow W^T of the 2-D encoder weights)
so clip_grad_norm_ + optimizer.step() (SURVEY.md K14+K15, ~1000 small launches) become 3 launches
with no host synchronisation. Elsewhere (CPU, or parameters outside a store) it falls back to the
exact torch.optim.Adam single-tensor math.
"""
from __future__ import annotations

import math
from typing import Iterable, Optional

import numpy as np
import torch

from .. import _ext



def _store_of(params):
    st = None
    for p in params:
        s = getattr(p, "_pvr_store_ref", None)
        s = s() if s is not None else None
        if s is None:
            return None
        if st is None:
            st = s
        elif s is not st:
            return None
    return st


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0,
                 decoupled_weight_decay: bool = False, skip_nonfinite: bool = True, amsgrad: bool = False,
                 maximize: bool = False):
        if amsgrad or maximize:
            raise NotImplementedError("FusedAdam supports neither amsgrad nor maximize")
        defaults = dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay,
                        decoupled_weight_decay=decoupled_weight_decay)
        super().__init__(params, defaults)
        self.skip_nonfinite = skip_nonfinite
        self._fused = None  # (store, m, v, seg_start, seg_group, ws, clip)
        self.last_grad_norm: Optional[torch.Tensor] = None
        self.step_count = 0
        # hipGraph mode: the per-step hyper-parameter table lives in a persistent device tensor that
        # graph_prepare() refreshes (outside the graph) before each replay
        self._graph = False
        self._table_dev: Optional[torch.Tensor] = None
        self._table_ring = []  # pinned host buffers + events (host may run a few steps ahead)
        self._ring_i = 0

    # ------------------------------------------------------------------ helpers
    def _all_params(self):
        return [p for g in self.param_groups for p in g["params"]]

    def _setup_fused(self):
        params = self._all_params()
        if not params or not params[0].is_cuda or not _ext.available():
            return None
        from ..runtime.param_store import lookup_store

        store = lookup_store(params[0])
        if store is None or any(lookup_store(p) is not store for p in params):
            return None
        if not all(store.covers_param(p) for p in params):
            return None
        fz = self._fused
        if fz is not None and fz[0] is store:
            return fz
        dev = store.device
        group_of = {}
        for gi, g in enumerate(self.param_groups):
            for p in g["params"]:
                group_of[id(p)] = gi
        starts, groups = [], []
        for p, off in zip(store.params, store.offsets):
            starts.append(off)
            groups.append(group_of.get(id(p), -1) if p.requires_grad else -1)
        seg_start = torch.tensor(starts, dtype=torch.int64, device=dev)
        seg_group = torch.tensor(groups, dtype=torch.int32, device=dev)
        m = torch.zeros(store.numel, dtype=torch.float32, device=dev)
        v = torch.zeros(store.numel, dtype=torch.float32, device=dev)
        # carry over any existing per-tensor state (e.g. loaded from a checkpoint)
        for p, off in zip(store.params, store.offsets):
            st = self.state.get(p)
            if st and "exp_avg" in st:
                m[off:off + p.numel()].copy_(st["exp_avg"].reshape(-1))
                v[off:off + p.numel()].copy_(st["exp_avg_sq"].reshape(-1))
                self.step_count = max(self.step_count, int(st.get("step", 0)))
        for p, off in zip(store.params, store.offsets):
            if id(p) in group_of:
                self.state[p] = {
                    "step": torch.tensor(float(self.step_count)),
                    "exp_avg": m[off:off + p.numel()].view(p.shape),
                    "exp_avg_sq": v[off:off + p.numel()].view(p.shape),
                }
        ws = torch.empty(_ext.ext().norm_partial_blocks(), dtype=torch.float32, device=dev)
        clip = torch.zeros(3, dtype=torch.float32, device=dev)
        self._fused = (store, m, v, seg_start, seg_group, ws, clip)
        self._tmeta_key = None
        return self._fused

    def _transposed_tables(self, store):
        """Tables of the fused Adam + W^T pass (csrc/optim.hip adam_t_kernel), rebuilt when the
        store's transposed layout changes; None if the store keeps no (64-aligned) W^T shadow."""
        lay = store.transposed_layout()
        if lay is None:
            return None
        tparams, tmeta_dev = lay
        key = (id(tmeta_dev), store.shadow_t.data_ptr())
        if self._tmeta_key == key:
            return self._ttables
        group_of = {}
        for gi, g in enumerate(self.param_groups):
            for p in g["params"]:
                group_of[id(p)] = gi
        meta = tmeta_dev.cpu().tolist()
        trows, tiles = [], 0
        for p, (soff, toff, R, C, _) in zip(tparams, meta):
            trows.append([soff, toff, R, C, tiles, group_of.get(id(p), -1) if p.requires_grad else -1])
            tiles += (R // 64) * (C // 64)
        tids = {id(p) for p in tparams}
        frows, f4 = [], 0
        for p, off in zip(store.params, store.offsets):
            if id(p) in tids:
                continue
            n = (p.numel() + 3) // 4 * 4  # the store pads every segment (zeros stay zero)
            frows.append([off, n, group_of.get(id(p), -1) if p.requires_grad else -1, f4])
            f4 += n // 4
        dev = store.device
        self._ttables = (torch.tensor(trows, dtype=torch.int64, device=dev), tiles,
                         torch.tensor(frows, dtype=torch.int64, device=dev), f4)
        self._tmeta_key = key
        return self._ttables

    def _group_array(self, step: int, arr: Optional[np.ndarray] = None) -> np.ndarray:
        G = len(self.param_groups)
        if arr is None:
            arr = np.zeros((G, 8), dtype=np.float32)
        for i, g in enumerate(self.param_groups):
            b1, b2 = g["betas"]
            arr[i, 0] = float(g["lr"])
            arr[i, 1] = b1
            arr[i, 2] = b2
            arr[i, 3] = g["eps"]
            arr[i, 4] = g["weight_decay"]
            arr[i, 5] = 1.0 - b1 ** step
            arr[i, 6] = math.sqrt(1.0 - b2 ** step)
        arr.view(np.int32)[:, 7] = [int(bool(g["decoupled_weight_decay"])) for g in self.param_groups]
        return arr

    def _group_table(self, step: int, device) -> torch.Tensor:
        if not self._graph:
            if len(self.param_groups) <= 8:
                # a host table travels in the launch's kernel arguments: no per-step H2D copy
                return torch.from_numpy(self._group_array(max(step, 1)))
            # same pinned-ring upload as the graph path: a pageable H2D copy would block the host until
            # the GPU queue drains (a ~0.3 ms bubble per step)
            if self._table_dev is None:
                self._alloc_table(device)
            self._upload_table(step)
        return self._table_dev

    def _alloc_table(self, device, ring: int = 4) -> None:
        G = len(self.param_groups)
        self._table_dev = torch.zeros(G, 8, dtype=torch.float32, device=device)
        self._table_ring = [(torch.zeros(G, 8, dtype=torch.float32).pin_memory(), torch.cuda.Event()) for _ in range(ring)]

    def _upload_table(self, step: int) -> None:
        host, ev = self._table_ring[self._ring_i % len(self._table_ring)]
        self._ring_i += 1
        ev.synchronize()  # the copy that last used this pinned buffer has executed
        self._group_array(max(step, 1), host.numpy())
        self._table_dev.copy_(host, non_blocking=True)
        ev.record()

    # ------------------------------------------------------------------ hipGraph support
    def graph_mode(self, enabled: bool = True, ring: int = 4) -> None:
        """Capture-safe stepping: ``step()`` reads the group table from a persistent device tensor and
        does not advance the step counter; call ``graph_prepare()`` before every graph replay."""
        fz = self._setup_fused()
        if enabled and fz is None:
            raise RuntimeError("graph mode needs the fused (single-store, GPU) optimizer path")
        self._graph = enabled
        if enabled:
            if self._table_dev is None:
                self._alloc_table(fz[0].device, ring)
            self.graph_prepare(advance=False)

    def graph_prepare(self, advance: bool = True) -> None:
        """Advance the step counter and upload this step's lr / bias corrections (stream-ordered)."""
        if advance:
            self.step_count += 1
        self._upload_table(self.step_count)

    # ------------------------------------------------------------------ public
    def zero_grad(self, set_to_none: bool = True):
        from ..runtime.param_store import lookup_store

        params = self._all_params()
        st = lookup_store(params[0]) if params else None
        if st is not None and all(lookup_store(p) is st for p in params):
            st.zero_grad()  # one memset, gradient views (= DDP buckets) stay attached
            return
        super().zero_grad(set_to_none=set_to_none)

    @torch.no_grad()
    def clip_grad_norm_(self, max_norm: float) -> torch.Tensor:
        """Global-norm clip of every gradient (after any DP all-reduce). Returns the norm (device)."""
        fz = self._setup_fused()
        if fz is None:
            params = [p for p in self._all_params() if p.grad is not None]
            n = torch.nn.utils.clip_grad_norm_(params, max_norm)
            self.last_grad_norm = n
            return n
        store, m, v, seg_start, seg_group, ws, clip = fz
        store.join_side()
        _ext.ext().grad_norm(store.grad_flat, float(max_norm), ws, clip)
        self._pending_clip = True
        self.last_grad_norm = clip[0]
        return clip[0]

    @torch.no_grad()
    def step(self, closure=None, clip_norm: Optional[float] = None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        fz = self._setup_fused()
        if not self._graph:
            self.step_count += 1
        step = self.step_count
        if fz is not None:
            store, m, v, seg_start, seg_group, ws, clip = fz
            store.join_side()  # weight gradients may still be in flight on the side stream
            use_clip = getattr(self, "_pending_clip", False)
            if clip_norm is not None:
                _ext.ext().grad_norm(store.grad_flat, float(clip_norm), ws, clip)
                self.last_grad_norm = clip[0]
                use_clip = True
            elif not use_clip and self.skip_nonfinite:
                _ext.ext().grad_norm(store.grad_flat, 0.0, ws, clip)  # max_norm 0 -> coef 1, flag only
                use_clip = True
            table = self._group_table(step, store.device)
            tt = self._transposed_tables(store)  # Adam also writes the bf16 W^T shadow when it can
            if tt is not None and tt[3] > 0:
                # master, m, v, bf16 shadow and the dgrad GEMMs' W^T shadow in one pass
                store.ensure_transposed()  # only if something else changed the weights since
                _ext.ext().adam_t(store.flat, store.grad_flat, m, v, store.shadow, store.shadow_t, tt[0], tt[1], tt[2], tt[3],
                                  table, clip if use_clip else None, self.skip_nonfinite)
                store.mark_shadow_fresh(transposed=True)
            else:
                _ext.ext().adam(store.flat, store.grad_flat, m, v, store.shadow, seg_start, seg_group, table,
                                clip if use_clip else None, self.skip_nonfinite)
                store.mark_shadow_fresh()
            self._pending_clip = False
            return loss
        # ---------------- reference math (torch.optim.Adam, single-tensor, maximize=False)
        if clip_norm is not None:
            self.clip_grad_norm_(clip_norm)
        for g in self.param_groups:
            b1, b2 = g["betas"]
            lr, eps, wd = g["lr"], g["eps"], g["weight_decay"]
            for p in g["params"]:
                if p.grad is None:
                    continue
                grad = p.grad
                st = self.state[p]
                if len(st) == 0 or "exp_avg" not in st:
                    st["step"] = torch.tensor(0.0)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["step"] += 1
                t = float(st["step"])
                if g["decoupled_weight_decay"]:
                    p.mul_(1 - lr * wd)
                elif wd != 0:
                    grad = grad.add(p, alpha=wd)
                st["exp_avg"].lerp_(grad, 1 - b1)
                st["exp_avg_sq"].mul_(b2).addcmul_(grad, grad.conj(), value=1 - b2)
                bc1 = 1 - b1 ** t
                bc2 = 1 - b2 ** t
                step_size = lr / bc1
                denom = (st["exp_avg_sq"].sqrt() / math.sqrt(bc2)).add_(eps)
                p.addcdiv_(st["exp_avg"], denom, value=-step_size)
        return loss

    def state_dict(self):
        if self._fused is not None:  # per-tensor step counters are materialised lazily
            for st in self.state.values():
                if "step" in st:
                    st["step"] = torch.tensor(float(self.step_count))
        return super().state_dict()

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        fz = self._fused
        self._fused = None
        if fz is not None:
            self._setup_fused()
