"""Operator layer: Python front-ends + autograd Functions over the gfx950 HIP kernels.

* ``gemm``      — MFMA GEMM forward / dgrad / wgrad with fused epilogues (csrc/gemm.hip)
* ``fused_vit`` — patch-embedding, encoder-block, head and cross-entropy autograd Functions
* ``functional``— single-op wrappers (layer_norm, attention) with PyTorch reference fallbacks
"""
from . import functional, gemm
from .fused_vit import cross_entropy

__all__ = ["gemm", "functional", "cross_entropy"]
