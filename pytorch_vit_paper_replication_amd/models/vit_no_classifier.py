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
        from ..ops.fused_vit import EncoderBlockFn, block_links, PatchEmbedFn, TokenLayerNormFn, site_drop
        from ..runtime.param_store import get_store

        c = self.config
        dev = x.device
        store = get_store(self, dev)
        store.refresh_shadow()
        if not getattr(store, "_vit_t_registered", False):
            store.register_transposed([w for blk in self.transformer_encoder for w in blk.fused_params()[2:12:2] if w.dim() == 2])
            store._vit_t_registered = True
        store.ensure_transposed()
        training = self.training
        store.grad_enabled = torch.is_grad_enabled()  # the fused Functions' forward runs with grad mode off
        if store.grad_enabled:
            store.prepare_grads()
        need_seed = training and (c["mlp_dropout"] > 0 or c["embedding_dropout"] > 0)
        seed = self._dropout_seed(dev) if need_seed else None
        pe = self.patch_embedding_block
        conv = pe.patch_and_flatten[0]
        tokens = PatchEmbedFn.apply(x, c["patch_size"], store, seed, pe.dropout.p, training,
                                    conv.weight, conv.bias, pe.class_token, pe.position_embedding)
        B, N = x.shape[0], pe.number_of_patches + 1
        f8 = self._fp8_state(dev, B * N)
        if f8 is not None:
            f8.begin_step(training)
        blocks = list(self.transformer_encoder)
        drops2 = [site_drop(seed, 2 + 2 * i, blk.mlp_block.mlp[4].p, training) for i, blk in enumerate(blocks)]
        links = block_links(blocks, drops2)
        for i, blk in enumerate(blocks):
            tokens = EncoderBlockFn.apply(tokens, B, N, blk.msa_block.multi_head_attention.num_heads,
                                          blk.msa_block.layer_norm.eps, blk.mlp_block.layer_norm.eps, store,
                                          site_drop(seed, 1 + 2 * i, blk.mlp_block.mlp[2].p, training), drops2[i],
                                          None if f8 is None else (f8, i), links[i], *blk.fused_params())
        y = TokenLayerNormFn.apply(tokens, self.layer_norm.eps, store, self.layer_norm.weight, self.layer_norm.bias)
        return y.float().view(B, N, -1)
