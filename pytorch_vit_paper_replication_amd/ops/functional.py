"""Single-op entry points: fused HIP kernel on GPU, PyTorch reference math elsewhere.

Useful for kernel tests and for building other models on the same kernels. Inputs on GPU are bf16
(activations) / fp32 (LayerNorm affine params); outputs follow the kernels' dtypes.
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch
import torch.nn.functional as F

from .. import _ext
from . import gemm as _g


def layer_norm(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor, eps: float = 1e-5) -> torch.Tensor:
    if _ext.use_fused(x) and x.dtype == torch.bfloat16:
        D = x.shape[-1]
        x2 = x.reshape(-1, D).contiguous()
        y, _, _ = _ext.ext().layernorm_fwd(x2, weight.float().contiguous(), bias.float().contiguous(), eps,
                                           x2.shape[0], D)
        return y.view_as(x)
    return F.layer_norm(x, (x.shape[-1],), weight, bias, eps)


def self_attention_qkv(qkv: torch.Tensor, batch: int, seq: int, heads: int) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    """Attention over a fused QKV projection ``[B*N, 3D]`` -> ``([B*N, D], lse [B*H, N] or None)``."""
    D = qkv.shape[1] // 3
    dh = D // heads
    if _ext.use_fused(qkv) and qkv.dtype == torch.bfloat16 and dh == 64:
        o, lse = _ext.ext().attn_fwd(qkv.contiguous(), batch, seq, heads, 1.0 / math.sqrt(dh))
        return o, lse
    q, k, v = qkv.view(batch, seq, 3, heads, dh).permute(2, 0, 3, 1, 4)
    o = F.scaled_dot_product_attention(q, k, v)
    return o.transpose(1, 2).reshape(batch * seq, D), None


def linear(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor] = None) -> torch.Tensor:
    if _ext.use_fused(x) and x.dtype == torch.bfloat16 and x.shape[-1] % 64 == 0 and w.shape[0] % 8 == 0:
        x2 = x.reshape(-1, x.shape[-1]).contiguous()
        y = _g.linear_fwd(x2, w.to(torch.bfloat16).contiguous(), None if b is None else b.float().contiguous())
        return y.view(*x.shape[:-1], w.shape[0])
    return F.linear(x, w, b)
