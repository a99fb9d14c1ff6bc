"""ViT backbone without the classifier head (reference models/vit_no_classifier.py:172-226).

``forward`` returns the final-LayerNorm'd full token sequence ``[B, N+1, D]``; the state_dict is the
full ViT's minus ``classifier.*``. The building blocks are shared with :mod:`.vit` (the reference keeps
verbatim copies; here there is one implementation).
"""
from __future__ import annotations

import torch
from torch import nn

from .. import _ext
from .vit import (MLPBlock, MultiHeadSelfAttentionBlock, PatchEmbedding, SelfAttention,  # noqa: F401
                  TransformerEncoderBlock, ViT as _FullViT)


class ViT(_FullViT):
    def __init__(self, image_size: int = 224, patch_size: int = 16, num_transformer_layer: int = 12,
                 num_heads: int = 12, embedding_dim: int = 768, mlp_size: int = 3072, attn_dropout: float = 0,
                 mlp_dropout: float = 0.1, embedding_dropout: float = 0.1):
        super().__init__(image_size=image_size, patch_size=patch_size, num_transformer_layer=num_transformer_layer,
                         num_heads=num_heads, embedding_dim=embedding_dim, mlp_size=mlp_size, attn_dropout=attn_dropout,
                         mlp_dropout=mlp_dropout, embedding_dropout=embedding_dropout, num_classes=1)
        del self.classifier
        self.config.pop("num_classes", None)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if _ext.use_fused(x) and self._fused_supported(x):
            return self._forward_fused_features(x)
        return self.forward_features(x)

    def _forward_fused_features(self, x: torch.Tensor) -> torch.Tensor:
        from ..ops.fused_vit import TokenLayerNormFn

        tokens, store, B, N = self._fused_encoder(x)  # the full ViT's fused encoder (device checks, side-stream join)
        y = TokenLayerNormFn.apply(tokens, self.layer_norm.eps, store, self.layer_norm.weight, self.layer_norm.bias)
        return y.float().view(B, N, -1)
