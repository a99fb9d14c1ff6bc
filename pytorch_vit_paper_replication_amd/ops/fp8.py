"""fp8 (OCP e4m3 / e5m2) GEMM path with per-tensor delayed scaling (SURVEY.md §7.2 step 9,
BASELINE.json config 5: ViT-H/14 fp8).

Recipe (the usual delayed-scaling scheme, all state on the device):
  * every quantized tensor has a slot: amax history (ring of ``history`` steps), quant scale
    ``qscale = fmax / max(history) * 2^-margin`` and dequant scale ``dscale = 1 / qscale``;
  * activations are quantized with the scale derived from PREVIOUS steps while the same pass
    records this step's amax; ``Fp8Meta.step()`` (once per training step, one kernel launch)
    rolls the histories. A slot seen for the first time is calibrated with one amax pass;
  * weights use current scaling (amax pass, then quantize) once per optimizer step, from the bf16
    shadow the fused Adam kernel already writes;
  * GEMMs run ``v_mfma_scale_f32_16x16x128_f8f6f4`` in the ping-pong kernel; the epilogue
    multiplies by ``dscale_a * dscale_b`` before bias / GELU / dropout / residual (csrc/gemm.hip).

Forward GEMMs use e4m3 x e4m3. With ``dgrad=True`` (``ViT.enable_fp8``'s default) the four
activation-gradient (dgrad) GEMMs of each encoder block also run in fp8: e5m2 gradients (own
delayed-scaling slots) x e4m3 transposed weights (``linear_dgrad_fp8``); with ``wgrad=True`` (also
the default) the four weight-gradient GEMMs too: e5m2 gradients^T x e4m3 activations^T from
transposing quantize passes (``linear_wgrad_fp8``, split-K over tokens). LayerNorm, softmax,
attention, residual adds and the optimizer stay in bf16 / fp32.
Non-finite values: an Inf element makes its tensor's amax non-finite and a NaN element propagates
through the NaN-aware amax reduction (csrc/fp8.hip); the scale update then leaves that slot's
history and scales unchanged, and FusedAdam's non-finite check skips the step.

Data parallelism: the amax histories and scales stay per rank, with no cross-rank max. A scale only
chooses how one rank's own activations / gradients are represented; every fp8 GEMM output is
dequantized in its epilogue, so the weight gradients that enter the all-reduce are plain fp32 values,
the averaged gradients are identical on every rank, and so are the global-norm clip, the non-finite
skip decision (taken on the all-reduced gradients: an overflow on one rank skips the step on all)
and the Adam update. Weight scales come from the weights themselves (current scaling), hence agree
across ranks. A cross-rank amax reduction would only matter for tensors sharded across ranks
(tensor / sequence parallelism), which this framework does not use. Pinned by
``tests/test_gpu_train.py::test_ddp_two_ranks_recipe`` (bitwise-equal parameters on both ranks after
every fp8 step, the overflowing step skipped on both).
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import torch

from .. import _ext
from . import gemm

E4M3, E5M2 = 0, 1
# fp8 weight gradients read the row-major fp8 copies directly (mn-contiguous GEMM operands); False:
# byte-transposed copies + the k-contiguous GEMM (test hook / A-B)
WGRAD_MN = True
FMAX = {E4M3: 448.0, E5M2: 57344.0}


class Fp8Meta:
    """Delayed-scaling state of ``n`` tensor slots."""

    def __init__(self, n: int, device, history: int = 16, margin: int = 0, fmt: int = E4M3):
        self.n = n
        self.fmt = fmt
        self.hist = torch.zeros(n, history, dtype=torch.float32, device=device)
        self.amax = torch.zeros(n, dtype=torch.int32, device=device)
        self.qscale = torch.ones(n, dtype=torch.float32, device=device)
        self.dscale = torch.ones(n, dtype=torch.float32, device=device)
        self.fmax = torch.full((n,), FMAX[fmt], dtype=torch.float32, device=device)
        self.margin_mul = 2.0 ** (-margin)
        self.calibrated = [False] * n

    def _update(self, s0: int, s1: int) -> None:
        _ext.ext().fp8_scale_update(self.hist, self.amax, self.qscale, self.dscale, self.fmax, s0, s1, self.margin_mul)

    def step(self) -> None:
        """Roll every slot's amax history into new scales (start of a training step)."""
        self._update(0, self.n)

    def quantize(self, x: torch.Tensor, slot: int, current: bool = False,
                 out: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
        """fp8 copy of a 2-D bf16 tensor -> (uint8 [rows, cols], dscale [1])."""
        ext = _ext.ext()
        am = self.amax[slot:slot + 1]
        if current or not self.calibrated[slot]:
            if current:  # current scaling: this tensor's amax alone (the last quantize pass recorded one)
                am.zero_()
            ext.fp8_quant(x, None, None, am, self.fmt)
            self._update(slot, slot + 1)
            self.calibrated[slot] = True
        y = out if out is not None else torch.empty(x.shape, dtype=torch.uint8, device=x.device)
        ext.fp8_quant(x, y, self.qscale[slot:slot + 1], am, self.fmt)
        return y, self.dscale[slot:slot + 1]

    def state_dict(self) -> Dict[str, torch.Tensor]:
        """Delayed-scaling state (CPU copies): amax histories, the running amax, both scales and the
        per-slot calibration flags; with it a resumed run quantizes exactly like the original."""
        return {"hist": self.hist.detach().cpu().clone(), "amax": self.amax.detach().cpu().clone(),
                "qscale": self.qscale.detach().cpu().clone(), "dscale": self.dscale.detach().cpu().clone(),
                "calibrated": torch.tensor(self.calibrated, dtype=torch.bool)}

    def load_state_dict(self, sd: Dict[str, torch.Tensor]) -> None:
        if tuple(sd["hist"].shape) != tuple(self.hist.shape):
            raise ValueError(f"fp8 state: history shape {tuple(sd['hist'].shape)} != {tuple(self.hist.shape)}")
        for k in ("hist", "amax", "qscale", "dscale"):
            getattr(self, k).copy_(sd[k].to(getattr(self, k).device))
        self.calibrated = [bool(v) for v in sd["calibrated"].tolist()]

    def producer(self, slot: int) -> Optional[Tuple["Fp8Meta", int]]:
        """(self, slot) if the slot is calibrated, so the kernel producing the tensor can write its fp8
        copy with the slot's delayed scale and record its amax (``quant=`` of the fp8 GEMMs); None on the
        tensor's first step, which goes through ``quantize`` (amax pass, then quantize)."""
        return (self, slot) if self.calibrated[slot] else None


class Fp8State:
    """Per-model fp8 state: activation slots (4 per encoder block) + weight cache."""

    ACT_PER_BLOCK = 4  # xn1 (qkv input), o (out-proj input), xn2 (fc1 input), h (fc2 input)

    def __init__(self, n_blocks: int, device, history: int = 16, margin: int = 0, dgrad: bool = True, wgrad: bool = True,
                 grad_fmt: int = E4M3):
        self.act = Fp8Meta(n_blocks * self.ACT_PER_BLOCK, device, history, margin, E4M3)
        # gradient slots for the fp8 dgrad GEMMs (dgrad=True): dz2, dU, dx1, dQKV per block; e4m3 by
        # default, e5m2 with grad_fmt=E5M2 (every producer of a gradient copy takes the slot's format)
        if grad_fmt not in (E4M3, E5M2):
            raise ValueError(f"Fp8State: grad_fmt {grad_fmt}")
        self.grad = Fp8Meta(n_blocks * self.ACT_PER_BLOCK, device, history, margin, grad_fmt)
        self.dgrad = bool(dgrad)
        self.wgrad = bool(wgrad) and bool(dgrad)  # fp8 weight gradients reuse the dgrad gradient slots
        self.n_blocks = n_blocks
        self._wmeta: Optional[Fp8Meta] = None
        self._wslot: Dict[int, int] = {}
        self._wcache: Dict[int, Tuple[int, torch.Tensor, torch.Tensor]] = {}
        self._wsrc: Dict[int, torch.Tensor] = {}   # key -> the bf16 shadow view it is quantized from
        self._batch: Optional[Tuple[torch.Tensor, int, int]] = None  # (segment table, chunks, keys)
        self._batch_gen: Optional[int] = None
        self._layout = None
        self.device = device

    def state_dict(self) -> Dict[str, Dict[str, torch.Tensor]]:
        """Activation / gradient slot state (weights use current scaling: nothing to keep)."""
        return {"act": self.act.state_dict(), "grad": self.grad.state_dict(), "grad_fmt": torch.tensor(self.grad.fmt)}

    def load_state_dict(self, sd) -> None:
        # the amax histories do not depend on the format (the scales are re-derived from them with the
        # slot's fmax at every step start), so a state from before the format field loads into either;
        # a recorded format must match for the resumed run to quantize like the original
        fmt = sd.get("grad_fmt")
        if fmt is not None and int(fmt) != self.grad.fmt:
            names = {E4M3: "e4m3", E5M2: "e5m2"}
            raise ValueError(f"fp8 state: saved with {names.get(int(fmt), fmt)} gradients, this model uses "
                             f"{names[self.grad.fmt]}: enable_fp8(grad_fmt='{names.get(int(fmt), fmt)}') to resume it")
        self.act.load_state_dict(sd["act"])
        self.grad.load_state_dict(sd["grad"])

    def begin_step(self, training: bool) -> None:
        if training:
            self.act.step()
            self.grad.step()

    def act_quant(self, x: torch.Tensor, block: int, which: int) -> Tuple[torch.Tensor, torch.Tensor]:
        return self.act.quantize(x, block * self.ACT_PER_BLOCK + which)

    def grad_quant(self, g: torch.Tensor, block: int, which: int) -> Tuple[torch.Tensor, torch.Tensor]:
        return self.grad.quantize(g, block * self.ACT_PER_BLOCK + which)

    def act_producer(self, block: int, which: int):
        return self.act.producer(block * self.ACT_PER_BLOCK + which)

    def grad_producer(self, block: int, which: int):
        return self.grad.producer(block * self.ACT_PER_BLOCK + which)

    def wgrad_ready(self, block: int, which_grad: int, which_act: int) -> bool:
        """fp8 weight gradient of (grad slot, activation slot) possible: both slots calibrated (the
        first step, which calibrates the gradient slots, computes its weight gradients in bf16)."""
        return (self.wgrad and self.grad.calibrated[block * self.ACT_PER_BLOCK + which_grad]
                and self.act.calibrated[block * self.ACT_PER_BLOCK + which_act])

    def linear_wgrad(self, dy: torch.Tensor, x: torch.Tensor, out: torch.Tensor, block: int, which_grad: int,
                     which_act: int, dy8: Optional[torch.Tensor] = None, x8: Optional[torch.Tensor] = None) -> torch.Tensor:
        n = self.ACT_PER_BLOCK
        return linear_wgrad_fp8(dy, self.grad, block * n + which_grad, x, self.act, block * n + which_act, out, dy8, x8)

    def weight(self, w16: torch.Tensor, key: int, generation: int, layout=None) -> Tuple[torch.Tensor, torch.Tensor]:
        """fp8 (e4m3, current scaling) copy of a bf16 weight shadow, cached per store generation.

        The first generation quantizes each weight on first use (two launches each) and records it;
        from then on a new generation re-quantizes EVERY recorded weight at once: one multi-tensor
        amax launch, one scale update, one multi-tensor quantize launch (instead of two launches per
        weight and direction, 512 per ViT-H/14 step).

        ``layout`` identifies the buffers every recorded source view lives in (the store's bf16 and
        transposed shadows): when it changes, the recorded views and the batched segment table are
        dropped, so no weight is ever re-quantized from a reallocated (stale) buffer."""
        if layout is not None and layout != self._layout:
            self._layout = layout
            self._wsrc.clear()
            self._wcache.clear()
            self._batch = None
            self._batch_gen = None
        hit = self._wcache.get(key)
        if hit is not None and hit[0] == generation:
            return hit[1], hit[2]
        src = self._wsrc.get(key)
        if (hit is not None and src is not None and src.data_ptr() == w16.data_ptr() and self._batch_gen != generation
                and w16.is_cuda and _ext.available()):
            self._refresh_all(generation)
            hit = self._wcache.get(key)
            if hit is not None and hit[0] == generation:
                return hit[1], hit[2]
        if key not in self._wslot:
            self._wslot[key] = len(self._wslot)
            if self._wmeta is None or self._wslot[key] >= self._wmeta.n:
                old = self._wmeta
                self._wmeta = Fp8Meta(max(64, 2 * len(self._wslot)), self.device, history=1, fmt=E4M3)
                if old is not None:  # grow: keep nothing (weights are re-scaled from scratch anyway)
                    self._wcache.clear()
        slot = self._wslot[key]
        out = hit[1] if hit is not None else None
        q, ds = self._wmeta.quantize(w16, slot, current=True, out=out)
        self._wcache[key] = (generation, q, ds)
        if self._wsrc.get(key) is None or self._wsrc[key].data_ptr() != w16.data_ptr():
            self._batch = None  # the recorded set changed: rebuild the segment table
        self._wsrc[key] = w16
        return q, ds

    def _refresh_all(self, generation: int) -> None:
        ext = _ext.ext()
        meta = self._wmeta
        keys = [k for k in self._wsrc if k in self._wcache]
        if self._batch is None or self._batch[2] != len(keys):
            rows, chunk0 = [], 0
            per = 256 * 16 * 4  # csrc/fp8.hip QM_CHUNK
            for k in keys:
                w16, q = self._wsrc[k], self._wcache[k][1]
                n = w16.numel()
                if n % 16 or w16.data_ptr() % 16 or q.data_ptr() % 16 or not (w16.is_contiguous() and q.is_contiguous()):
                    return  # not batchable (16-B vector accesses): the per-weight path handles this generation
                rows.append([w16.data_ptr(), q.data_ptr(), n, self._wslot[k], chunk0])
                chunk0 += (n + per - 1) // per
            self._batch = (torch.tensor(rows, dtype=torch.int64, device=self.device), chunk0, len(keys))
        segs, nchunks, _ = self._batch
        # current scaling: each weight's scale from its own amax now (the quantize pass of the previous
        # generation left its amax recorded, which would make the scale depend on the last two weights)
        meta.amax.zero_()
        ext.fp8_quant_multi(segs, nchunks, None, meta.amax, E4M3, True)
        meta._update(0, meta.n)
        ext.fp8_quant_multi(segs, nchunks, meta.qscale, meta.amax, E4M3, False)
        for k in keys:
            _, q, ds = self._wcache[k]
            self._wcache[k] = (generation, q, ds)
        self._batch_gen = generation


def _quant_args(quant, rows: int, cols: int, device):
    """``quant=(meta, slot)`` of the fp8 GEMMs -> (gemm_fp8 kwargs, (fp8 copy, dequant scale))."""
    if quant is None:
        return {}, None
    meta, slot = quant
    q = torch.empty(rows, cols, dtype=torch.uint8, device=device)
    kw = dict(q_out=q, q_scale=meta.qscale[slot:slot + 1], q_amax=meta.amax[slot:slot + 1], q_fmt=meta.fmt)
    return kw, (q, meta.dscale[slot:slot + 1])


def layernorm_fwd_q8(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, eps: float, quant, skip_y: bool = False):
    """LayerNorm forward that also writes the output's e4m3 copy with a calibrated slot's delayed scale
    (``quant=(meta, slot)``, ``Fp8Meta.producer``) and records its amax:
    returns ``(y, mean, rstd, (y_fp8, dequant scale))``."""
    meta, slot = quant
    T, D = x.shape
    q = torch.empty(T, D, dtype=torch.uint8, device=x.device)
    y, mean, rstd = _ext.ext().layernorm_fwd_q8(x, w, b, eps, T, D, q, meta.qscale[slot:slot + 1], meta.amax[slot:slot + 1],
                                                bool(skip_y))
    return y, mean, rstd, (q, meta.dscale[slot:slot + 1])


def linear_fwd_fp8(xq: torch.Tensor, xs: torch.Tensor, wq: torch.Tensor, ws: torch.Tensor,
                   bias: Optional[torch.Tensor] = None, *, resid: Optional[torch.Tensor] = None, drop=None,
                   gelu_aux: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None, quant=None,
                   skip_out: bool = False, gelu: bool = False):
    """y = resid + dropout(dequant(xq . wq^T) + bias), or the GELU variant (see gemm.linear_fwd).

    ``quant=(meta, slot)`` (GELU variant, a calibrated slot: ``Fp8Meta.producer``): the epilogue also
    writes y's fp8 copy with the slot's delayed scale and records y's amax, so the next GEMM needs no
    quantize pass; returns ``(y, (y_fp8, dequant scale))`` then. ``skip_out`` (with ``quant``): the bf16
    y is not stored (allocated, unwritten) - for when every consumer reads the fp8 copy. ``gelu=True``
    without ``gelu_aux``: the GELU epilogue for inference (no derivative stored)."""
    T, K = xq.shape
    N = wq.shape[0]
    if out is None:
        out = torch.empty(T, N, dtype=torch.bfloat16, device=xq.device)
    seed, soff, p = gemm._drop_args(drop)
    epi = gemm.EPI_GELU if (gelu or gelu_aux is not None) else gemm.EPI_BF16
    kw, q = _quant_args(quant, T, N, xq.device)
    _ext.ext().gemm_fp8(xq, E4M3, wq, E4M3, out, T, N, K, epi, xs, ws, bias, resid, gelu_aux, seed, soff, p,
                        c_skip=bool(skip_out and quant is not None), **kw)
    return out if quant is None else (out, q)


def linear_dgrad_fp8(gq: torch.Tensor, gs: torch.Tensor, wtq: torch.Tensor, wts: torch.Tensor, *,
                     dgelu_aux: Optional[torch.Tensor] = None, colsum: Optional[torch.Tensor] = None,
                     out: Optional[torch.Tensor] = None, quant=None, skip_out: bool = False, g_fmt: int = E5M2):
    """dx = dequant(gq (e5m2, or e4m3: ``g_fmt``) . wtq^T (e4m3, W^T rows)) [* dgelu_aux]; ``quant`` as in
    linear_fwd_fp8 (dGELU variant: the gradient-format copy of dx for the next dgrad GEMM)."""
    T, N = gq.shape
    K = wtq.shape[0]
    if out is None:
        out = torch.empty(T, K, dtype=torch.bfloat16, device=gq.device)
    epi = gemm.EPI_DGELU if dgelu_aux is not None else gemm.EPI_BF16
    kw, q = _quant_args(quant, T, K, gq.device)
    _ext.ext().gemm_fp8(gq, g_fmt, wtq, E4M3, out, T, K, N, epi, gs, wts, None, None, dgelu_aux, None, 0, 0.0, colsum,
                        c_skip=bool(skip_out and quant is not None), tail_limit=gemm.DGRAD_TAIL_UNITS, **kw)
    return out if quant is None else (out, q)


def linear_wgrad_fp8(dy: torch.Tensor, dy_meta: "Fp8Meta", dy_slot: int, x: torch.Tensor, x_meta: "Fp8Meta", x_slot: int,
                     out: torch.Tensor, dy8: Optional[torch.Tensor] = None, x8: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out[N, K] += dequant(dy^T (the gradient slot's format, e5m2 or e4m3) . x (e4m3)) over the tokens:
    the weight gradient in fp8.

    Both operands are needed TRANSPOSED ([features][tokens], the token dim padded to 128 with zeros)
    with their slots' current delayed scales. ``dy8`` / ``x8``: the row-major fp8 copies the dgrad /
    forward GEMMs already used (same slots, same scales) -> a byte transpose (1 byte read per
    element); otherwise a transposing quantize pass over the bf16 tensor (the slots' amax is recorded
    by the non-transposed passes). Then the k-contiguous fp8 ping-pong GEMM runs split-K over tokens
    into a workspace, reduced into ``out`` in a fixed order (deterministic)."""
    ext = _ext.ext()
    T, N = dy.shape
    K = x.shape[1]
    if dy8 is not None and x8 is not None and WGRAD_MN:
        # both row-major copies exist: the GEMM reads them as mn-contiguous operands (no transposes)
        splits = gemm.wgrad_splits(T, N, K, 12)
        ksplit = max(128, (T // splits + 127) // 128 * 128)
        nsplit = (T + ksplit - 1) // ksplit
        ws = gemm._workspace(nsplit * N * K, dy.device)[:nsplit * N * K].view(nsplit, N, K)
        ext.gemm_fp8_wgrad_mn(dy8, x8, ws, N, K, T, dy_meta.dscale[dy_slot:dy_slot + 1], x_meta.dscale[x_slot:x_slot + 1], ksplit,
                              dy_meta.fmt)
        ext.splitk_reduce(ws, nsplit, out, True)
        return out
    Tp = (T + 127) // 128 * 128
    dyt = torch.empty(N, Tp, dtype=torch.uint8, device=dy.device)
    xt = torch.empty(K, Tp, dtype=torch.uint8, device=dy.device)
    if dy8 is not None:
        ext.fp8_transpose(dy8, dyt)
    else:
        ext.fp8_quant_t(dy, dyt, dy_meta.qscale[dy_slot:dy_slot + 1], dy_meta.fmt)
    if x8 is not None:
        ext.fp8_transpose(x8, xt)
    else:
        ext.fp8_quant_t(x, xt, x_meta.qscale[x_slot:x_slot + 1], E4M3)
    splits = gemm.wgrad_splits(T, N, K, 12)
    ksplit = max(128, (Tp // splits + 127) // 128 * 128)
    nsplit = (Tp + ksplit - 1) // ksplit
    ws = gemm._workspace(nsplit * N * K, dy.device)[:nsplit * N * K].view(nsplit, N, K)
    ext.gemm_fp8_wgrad(dyt, xt, ws, N, K, Tp, dy_meta.dscale[dy_slot:dy_slot + 1], x_meta.dscale[x_slot:x_slot + 1], ksplit,
                       dy_meta.fmt)
    ext.splitk_reduce(ws, nsplit, out, True)
    return out


def supported(T: int, D: int, M: int) -> bool:
    return D % 128 == 0 and M % 128 == 0 and T >= 256
