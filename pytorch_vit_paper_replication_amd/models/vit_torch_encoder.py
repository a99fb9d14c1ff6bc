"""ViT built on ``torch.nn.TransformerEncoder`` (the reference's exercise 1).

The exercise notebook (EX.ipynb:535-598) swaps the hand-written encoder blocks for
``nn.TransformerEncoderLayer(norm_first=True, activation="gelu", batch_first=True)`` stacked by
``nn.TransformerEncoder(..., norm=LayerNorm)``; same parameter count as the custom ViT (85,800,963
for 3 classes, EX.ipynb:662) but different state_dict names. Two deliberate differences:

  * the notebook passes ``num_layers=num_heads`` (EX.ipynb:579), a bug masked because both are 12;
    here ``num_transformer_layer`` is honoured (``replicate_num_layers_bug=True`` restores the
    notebook's behaviour);
  * ``to_vit()`` converts the model into this framework's ``ViT`` (identical eval-mode math: pre-LN
    blocks, erf-GELU, final LayerNorm, CLS head), so a prototype trained this way runs on the fused
    MI355X kernels. The converse, ``from_vit()``, loads a ``ViT`` state_dict into the prototype. In
    training mode the layers differ in dropout placement only: ``TransformerEncoderLayer`` also
    drops the attention output and the attention probabilities, the reference blocks do not
    (reference models/vit.py:167).
"""
from __future__ import annotations

from typing import Dict

import torch
from torch import nn

from .vit import PatchEmbedding, ViT


class ViTTorchEncoder(nn.Module):
    def __init__(self, image_size: int = 224, patch_size: int = 16, num_transformer_layer: int = 12,
                 num_heads: int = 12, embedding_dim: int = 768, mlp_size: int = 3072, mlp_dropout: float = 0.1,
                 embedding_dropout: float = 0.1, num_classes: int = 1000, replicate_num_layers_bug: bool = False):
        super().__init__()
        self.patch_embedding_block = PatchEmbedding(image_size=image_size, patch_size=patch_size,
                                                    embedding_dim=embedding_dim, embedding_dropout=embedding_dropout)
        layer = nn.TransformerEncoderLayer(d_model=embedding_dim, nhead=num_heads, dim_feedforward=mlp_size,
                                           dropout=mlp_dropout, activation="gelu", batch_first=True, norm_first=True)
        self.transformer_encoder = nn.TransformerEncoder(
            encoder_layer=layer, num_layers=num_heads if replicate_num_layers_bug else num_transformer_layer,
            norm=nn.LayerNorm(embedding_dim), enable_nested_tensor=False)
        self.classifier = nn.Sequential(nn.Linear(in_features=embedding_dim, out_features=num_classes))
        self.config = dict(image_size=image_size, patch_size=patch_size,
                           num_transformer_layer=len(self.transformer_encoder.layers), num_heads=num_heads,
                           embedding_dim=embedding_dim, mlp_size=mlp_size, attn_dropout=mlp_dropout,
                           mlp_dropout=mlp_dropout, embedding_dropout=embedding_dropout, num_classes=num_classes)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = self.patch_embedding_block(x)
        x = self.transformer_encoder(x)
        return self.classifier(x[:, 0])

    # ------------------------------------------------------------------ conversion
    _LAYER = {
        "self_attn.in_proj_weight": "msa_block.multi_head_attention.in_proj_weight",
        "self_attn.in_proj_bias": "msa_block.multi_head_attention.in_proj_bias",
        "self_attn.out_proj.weight": "msa_block.multi_head_attention.out_proj.weight",
        "self_attn.out_proj.bias": "msa_block.multi_head_attention.out_proj.bias",
        "linear1.weight": "mlp_block.mlp.0.weight",
        "linear1.bias": "mlp_block.mlp.0.bias",
        "linear2.weight": "mlp_block.mlp.3.weight",
        "linear2.bias": "mlp_block.mlp.3.bias",
        "norm1.weight": "msa_block.layer_norm.weight",
        "norm1.bias": "msa_block.layer_norm.bias",
        "norm2.weight": "mlp_block.layer_norm.weight",
        "norm2.bias": "mlp_block.layer_norm.bias",
    }

    def vit_state_dict(self) -> Dict[str, torch.Tensor]:
        out = {}
        for k, v in self.state_dict().items():
            if k.startswith("transformer_encoder.layers."):
                _, _, i, rest = k.split(".", 3)
                out[f"transformer_encoder.{i}.{self._LAYER[rest]}"] = v
            elif k.startswith("transformer_encoder.norm."):
                out["layer_norm." + k.rsplit(".", 1)[1]] = v
            else:
                out[k] = v
        return out

    def to_vit(self) -> ViT:
        """An equivalent framework ``ViT`` (attention dropout = the layer's dropout, as in the layer)."""
        c = dict(self.config)
        vit = ViT(**c)
        vit.load_state_dict(self.vit_state_dict(), strict=True)
        return vit.to(next(self.parameters()).device)

    def from_vit(self, vit: ViT) -> "ViTTorchEncoder":
        inv = {v: k for k, v in self._LAYER.items()}
        sd = {}
        for k, v in vit.state_dict().items():
            if k.startswith("transformer_encoder."):
                _, i, rest = k.split(".", 2)
                sd[f"transformer_encoder.layers.{i}.{inv[rest]}"] = v
            elif k.startswith("layer_norm."):
                sd["transformer_encoder.norm." + k.split(".", 1)[1]] = v
            else:
                sd[k] = v
        self.load_state_dict(sd, strict=True)
        return self
