"""Python front-end of the MFMA GEMM (csrc/gemm.hip): forward / dgrad / wgrad of a Linear layer.

Shapes follow nn.Linear: ``x [T, K]``, ``w [N, K]`` (bf16 shadow of the fp32 master weight),
``y = x . w^T [T, N]``. All three products run on the same hand-written kernel template with
different operand layouts (k-contiguous or mn-contiguous LDS staging) — there are no transposed
copies of activations or weights anywhere.
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch

from .. import _ext

EPI_BF16, EPI_GELU, EPI_DGELU, EPI_F32_ATOMIC, EPI_F32_STORE = range(5)

# tile configs (csrc/gemm.hip): 0 = 128x128 (4 waves), 6 = 256x256 BK=32 ring, 12 = 256x256 8-wave
# ping-pong, 13 = its persistent form, 14 = ping-pong with split-K f32 partial stores


def _n_cus() -> int:
    global _N_CUS
    if _N_CUS is None:
        _N_CUS = torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count if torch.cuda.is_available() else 256
    return _N_CUS


_N_CUS = None
# test hook (tests/kernel_checks.py): force one tile config for every GEMM while set
FORCE_TILE: Optional[int] = None

Drop = Optional[Tuple[torch.Tensor, int, float]]  # (int64 seed tensor on device, site offset, p)


def _tile(M: int, N: int, K: int, kind: str) -> int:
    """Tile config per GEMM kind (measured on MI355X, scripts/bench_kernels.py, profiles/):
    k-contiguous forward/dgrad at ViT sizes -> 256x256 8-wave ping-pong, persistent (13) when there
    are at least four output tiles per CU, one tile per workgroup (12) otherwise (K % 64 != 0: the
    4-stage BK=32 ring, 6); token-reduced wgrad (both operands mn-contiguous, split-K) -> the same
    ping-pong with transposed LDS reads when the token count is large, 128x128 (0) otherwise."""
    if FORCE_TILE is not None:
        return int(FORCE_TILE)
    if kind in ("fwd", "dgrad_t") and M >= 2048 and N >= 256:
        if K % 64:
            return 6
        # persistent ping-pong (13): the next tile's K-tiles stream in under this tile's epilogue.
        # It pays for the VALU-heavy GELU epilogue (fc1 fwd 0.377 vs 0.457 ms at ViT-B/16 b256,
        # profiles/kbench_epilogues.log); epilogues that load per-row inputs (residual, dGELU
        # factor) drain the in-flight DMAs there and stay on the one-tile-per-workgroup form (12).
        # persistent ping-pong (13) once there are at least four tiles per CU: the next tile's
        # K-tiles stream in under the register-direct epilogue, whose stores stay in flight under
        # the next tile's first K-tile (qkv fwd 0.171-0.179 vs 0.183-0.185 ms, fc1 GELU fwd 0.347-0.352
        # vs 0.361-0.367; N = 768 (2.3 tiles per CU) neutral: profiles/r3/ppp_direct_ab.log). The dGELU
        # dgrad (column-sum exchange at every tile end) too since round 5: 0.298-0.303 vs 0.311-0.315 ms
        # with the column sums (profiles/r5/tiles_12_13/; round 3 measured the opposite before the
        # register-direct epilogues, profiles/r3/gemm_ab.log)
        # K <= 2048 only: at ViT-L/16-384 (T = 73,856, N = 1024: 4.5 tiles per CU) the long-K GEMMs run
        # faster one tile per workgroup (fc2 fwd K 4096 0.520 vs 0.539 ms, qkv dgrad K 3072 0.380 vs
        # 0.396, fc1 dgrad 0.503 vs 0.510; profiles/r5/tiles_12_13/l16_ab.log; ViT-B/16 has no such
        # GEMM above four tiles per CU, hence round 4's "no gain", profiles/r4/pmaxk/)
        if 128 <= K <= 2048 and math.ceil(M / 256) * math.ceil(N / 256) >= 4 * _n_cus():
            return 13
        return 12
    if kind == "wgrad" and K >= 4096 and M >= 256 and N >= 256:
        return 12
    return 0


# Wave-specialized persistent kernel (tile 15, csrc/gemm_ws.hip: 8 MFMA waves + 8 epilogue waves per
# CU, the epilogue of tile t - 2 running beside the MFMAs of tile t) for these GEMM kinds of the
# large-token path: "gelu" (fc1 forward: GELU + dropout + derivative), "dgelu" (fc2 dgrad: x dGELU
# factor + bias-gradient column sums), "bias" (qkv forward), "resid" (out-proj / fc2 forward: dropout +
# residual), "dgrad" (plain dgrads). PVR_GEMM_WS=kind,kind overrides (empty: none).
import os as _os

WS_KINDS = set(k for k in _os.environ.get("PVR_GEMM_WS", "").split(",") if k)


def _ws_tile(kind: str, t: int) -> int:
    """Tile 15 for a GEMM kind routed to the wave-specialized kernel, where the default choice is a
    256x256 ping-pong one (12 / 13); the kernel itself falls back to tile 13 for shapes it cannot take."""
    if FORCE_TILE is None and kind in WS_KINDS and t in (12, 13):
        return 15
    return t


def _small_splitk(T: int, N: int, K: int) -> int:
    """K splits for a forward GEMM on 256x256 tiles (T >= 2048) with fewer than 128 output tiles
    (0: do not split). Each split keeps at least two 64-deep K-tiles; the splits aim at ~256
    workgroups. Measured (profiles/r2s/small_splitk_ab.log): eval forward at batch 32 +5 %; below
    2048 rows the 128x128 one-pass tiles are faster (batch 1: 1.32 ms unsplit vs 1.89 split)."""
    if K % 128 or N % 4 or T < 2048:
        return 0
    tiles = math.ceil(T / 256) * math.ceil(N / 256)
    if tiles >= 128:
        return 0
    s = min(K // 128, max(2, 256 // tiles))
    return s if s >= 2 else 0


# Split-K tail of the last dispatch round (csrc/gemm.hip plan_tail): forward GEMMs take it without a
# limit (nothing runs beside them); the backward's dgrad GEMMs only when the split round stays this
# small, because the weight-gradient side stream's long workgroups hold the CUs a wide split round
# needs (ViT-B/16 b256: unlimited -0.6 % per step, profiles/r4/tail_ab.md). -1 disables (A/B).
DGRAD_TAIL_UNITS = 64


def _gemm(*args, tile: int, colsum=None, tail_limit: int = 0):
    _ext.ext().gemm(*args, tile, colsum=colsum, tail_limit=tail_limit)


def _drop_args(drop: Drop):
    if drop is None or drop[2] <= 0.0:
        return None, 0, 0.0
    return drop[0], int(drop[1]), float(drop[2])


def linear_fwd(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None, *,
               resid: Optional[torch.Tensor] = None, drop: Drop = None, gelu_aux: Optional[torch.Tensor] = None,
               gelu: bool = False,
               addend: Optional[torch.Tensor] = None, addend_period: int = 0,
               row_remap: Tuple[int, int, int] = (0, 0, 0), out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """y = resid + dropout(x.w^T + bias + addend[row % period]).

    GELU variant (``gelu_aux`` given): u = x.w^T + bias, y = dropout(gelu(u)) and gelu_aux receives
    mask * scale * gelu'(u) — exactly the factor ``linear_dgrad(..., dgelu_aux=)`` multiplies by.
    ``gelu=True`` without ``gelu_aux``: the GELU epilogue for inference (no derivative stored)."""
    T, K = x.shape
    N = w.shape[0]
    if out is None:
        out = torch.empty(T, N, dtype=torch.bfloat16, device=x.device)
    seed, soff, p = _drop_args(drop)
    epi = EPI_GELU if (gelu or gelu_aux is not None) else EPI_BF16
    S = _small_splitk(T, N, K) if (p == 0.0 and gelu_aux is None and addend is None and row_remap[0] == 0) else 0
    if S:
        # serving-size batch: split K over workgroups (fp32 partials, tile 14), then one pass sums
        # them and applies bias / GELU / residual
        ksplit = math.ceil(math.ceil(K / S) / 64) * 64
        nsplit = math.ceil(K / ksplit)
        ws = _workspace(nsplit * T * N, x.device)[:nsplit * T * N].view(nsplit, T, N)
        ext = _ext.ext()
        ext.gemm(x, True, w, True, ws, T, N, K, EPI_F32_STORE, None, None, None, 0, None, 0, 0, 0, None, 0, 0.0, ksplit, 14)
        ext.splitk_epilogue(ws, nsplit, out, bias, resid, epi == EPI_GELU)
        return out
    kind = "gelu" if epi == EPI_GELU else "resid" if resid is not None else "bias"
    _gemm(x, True, w, True, out, T, N, K, epi, bias, resid, addend, addend_period, gelu_aux,
          row_remap[0], row_remap[1], row_remap[2], seed, soff, p, 0,
          tile=_ws_tile(kind, _tile(T, N, K, "fwd")) if addend is None and row_remap[0] == 0 else _tile(T, N, K, "fwd"))
    return out


def linear_dgrad(dy: torch.Tensor, w: torch.Tensor, *, dgelu_aux: Optional[torch.Tensor] = None,
                 drop: Drop = None, out: Optional[torch.Tensor] = None, wt: Optional[torch.Tensor] = None,
                 colsum: Optional[torch.Tensor] = None, tile: Optional[int] = None) -> torch.Tensor:
    """dx = dy . w ; optionally fused with the GELU + dropout backward of the producing layer:
    dx = (dy . w) * dgelu_aux (the factor saved by the GELU forward epilogue). With ``wt`` (= w^T, [K, N] bf16) the weight operand is
    k-contiguous and the fast forward-layout kernel runs; otherwise w is read with transposed LDS reads."""
    T, N = dy.shape
    K = w.shape[1]
    if out is None:
        out = torch.empty(T, K, dtype=torch.bfloat16, device=dy.device)
    seed, soff, p = None, 0, 0.0  # the mask is already folded into dgelu_aux
    epi = EPI_DGELU if dgelu_aux is not None else EPI_BF16
    if colsum is not None and dgelu_aux is None:
        raise ValueError("colsum is fused only into the GELU-backward epilogue")
    if wt is not None and N % 64 == 0:
        _gemm(dy, True, wt, True, out, T, K, N, epi, None, None, None, 0, dgelu_aux, 0, 0, 0,
              seed, soff, p, 0, tile=_ws_tile("dgelu" if dgelu_aux is not None else "dgrad", _tile(T, K, N, "dgrad_t")),
              colsum=colsum, tail_limit=DGRAD_TAIL_UNITS)
    else:
        _ext.ext().gemm(dy, True, w, False, out, T, K, N, epi, None, None, None, 0, dgelu_aux, 0, 0, 0,
                        seed, soff, p, 0, _tile(T, K, N, "dgrad") if tile is None else tile, colsum=colsum,
                        tail_limit=DGRAD_TAIL_UNITS)
    return out


# workgroups a 256x256 weight-gradient GEMM is split into: one resident workgroup per CU (measured
# best beside the dgrad chain, scripts/gpu_wgs_ab.sh in round 2)
_WGRAD_WGS = 256
_WGRAD_WGS_NARROW = 144
OVERLAPPED = False  # set by ParamStore.on_side while it launches side-stream weight gradients


def wgrad_splits(T: int, N: int, K: int, tile: int = 0) -> int:
    """Token splits of a weight-gradient GEMM (each split accumulates into dW with f32 atomics).
    256x256 ping-pong tiles (12): one resident workgroup per CU, so fill the 256 CUs once, except
    for the narrow weights of a 768-wide model (their 9-36 tiles would take 7-28 splits) while they
    run on the side stream (OVERLAPPED): ~144 workgroups there, leaving CUs to the dgrads they
    overlap with on the main stream (ViT-B/16 b256 +0.8-1.0 %; ViT-L/16 and ViT-H/14 lose 1 % with
    it; profiles/r5/wgrad_width/); 128x128 tiles (0): about 1024 workgroups."""
    if tile == 12:
        tiles = math.ceil(N / 256) * math.ceil(K / 256)
        wgs = _WGRAD_WGS_NARROW if OVERLAPPED and min(N, K) <= 768 else _WGRAD_WGS
        return max(1, min(wgs // tiles, max(1, T // 256)))
    tiles = math.ceil(N / 128) * math.ceil(K / 128)
    target = 1024
    s = max(1, round(target / tiles))
    s = min(s, max(1, T // 512))
    return s


# in-launch split-K reduction of the weight gradients (GemmParams::sk_*), opt-in (PVR_SPLITK_FIXUP=1):
# measured slower than the separate splitk_reduce pass at every ViT-B/16 shape (fc1 0.253 vs 0.239 ms,
# out 0.100 vs 0.084; b256 step 7384 vs 7439 img/s; profiles/r6/splitk/): each split's write-through
# slab drain, the wait for its siblings and its 256 KiB of sc1 reads run at one CU's bandwidth,
# while the separate pass streams every slab at full-chip bandwidth
SPLITK_FIXUP = _os.environ.get("PVR_SPLITK_FIXUP", "0") != "0"
_cus = None


def _num_cus() -> int:
    global _cus
    if _cus is None:
        _cus = int(_ext.ext().num_cus())
    return _cus


_workspaces = {}  # (device index, stream id) -> flat f32 split-K workspace


def _workspace(numel: int, device: torch.device) -> torch.Tensor:
    """Split-K partial buffer, one per (device, stream): weight-gradient GEMMs on one stream are
    serialised, so they can share it; grown (never shrunk) to the largest request."""
    key = (device.index, torch.cuda.current_stream(device).stream_id)
    ws = _workspaces.get(key)
    if ws is None or ws.numel() < numel:
        ws = torch.empty(numel, dtype=torch.float32, device=device)
        _workspaces[key] = ws
    return ws


def linear_wgrad(dy: torch.Tensor, x: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
    """out[N, K] += dy^T . x   (fp32, split over tokens).

    ``out`` may be narrower than x ([N, K'] with K' < K, K' % 4 == 0): it receives the first K'
    columns (the patch embedding's K, padded to the GEMM tile in x, reduced into the unpadded
    weight gradient without a temporary).

    Large token counts (tile 12/14 ping-pong) write each split's partial product to a workspace with
    LDS-staged coalesced stores, then one reduction pass adds the slices into ``out`` in a fixed
    order. That is 8-25 % faster than f32 atomics at ViT-B/16 shapes (the L2 executes atomics one
    element at a time, profiles/wgrad_epilogue_ab.log) and makes the weight gradients deterministic.
    Small GEMMs accumulate with f32 atomics."""
    T, N = dy.shape
    K = x.shape[1]
    tile = _tile(N, K, T, "wgrad")
    splits = wgrad_splits(T, N, K, tile)
    if tile != 12 and splits > 1 and _ext.deterministic():
        splits = 1  # the atomic path: one token range, so one add per element (deterministic)
    ksplit = math.ceil(math.ceil(T / splits) / 64) * 64
    ext = _ext.ext()
    nsplit = math.ceil(T / ksplit)
    narrow = out.shape[-1] < K
    # the split-K reduction writes 16-B column groups: a narrow out needs a width % 4 == 0 (odd
    # patch sizes, kc = 3 * P * P odd, take the temporary below)
    if tile == 12 and nsplit > 1 and out.is_contiguous() and N % 4 == 0 and out.shape[-1] % 4 == 0:
        ws = _workspace(nsplit * N * K, dy.device)[:nsplit * N * K].view(nsplit, N, K)
        if SPLITK_FIXUP and not narrow and math.ceil(N / 256) * math.ceil(K / 256) * nsplit <= _num_cus():
            # in-launch reduction: each split adds 1/nsplit of its tile, summed over the slabs in a
            # fixed order, into out (no separate reduce pass; deterministic)
            ext.gemm(dy, False, x, False, ws, N, K, T, EPI_F32_STORE, None, None, None, 0, None, 0, 0, 0,
                     None, 0, 0.0, ksplit, 14, reduce_out=out, reduce_acc=True)
            return out
        ext.gemm(dy, False, x, False, ws, N, K, T, EPI_F32_STORE, None, None, None, 0, None, 0, 0, 0,
                 None, 0, 0.0, ksplit, 14)
        ext.splitk_reduce(ws, nsplit, out, True)
        return out
    if nsplit > 1 and _ext.deterministic():
        # the f32-atomic epilogue below adds every token split into the same element: one split only
        ksplit, nsplit = math.ceil(T / 64) * 64, 1
    if narrow:
        tmp = torch.zeros(N, K, dtype=torch.float32, device=dy.device)
        linear_wgrad(dy, x, tmp)
        out.add_(tmp[:, :out.shape[-1]])
        return out
    ext.gemm(dy, False, x, False, out, N, K, T, EPI_F32_ATOMIC, None, None, None, 0, None, 0, 0, 0,
             None, 0, 0.0, ksplit, tile)
    return out


def bias_grad(dy: torch.Tensor, db: Optional[torch.Tensor], *, drop: Drop = None,
              dz: Optional[torch.Tensor] = None, quant=None):
    """db += column sums of (mask * dy); writes the masked gradient to dz when given.

    ``quant=(meta, slot)`` (a calibrated gradient slot, ``Fp8Meta.producer``): the same pass writes the
    (masked) gradient's fp8 copy in the slot's format with the slot's delayed scale and records its amax; returns
    ``(copy, dequant scale)`` then."""
    T, N = dy.shape
    seed, soff, p = _drop_args(drop)
    if quant is None:
        _ext.ext().colsum(dy, T, N, db, dz, seed, soff, p)
        return None
    meta, slot = quant
    q = torch.empty(T, N, dtype=torch.uint8, device=dy.device)
    _ext.ext().colsum(dy, T, N, db, dz, seed, soff, p, q_out=q, q_scale=meta.qscale[slot:slot + 1],
                      q_amax=meta.amax[slot:slot + 1], q_fmt=meta.fmt)
    return q, meta.dscale[slot:slot + 1]
