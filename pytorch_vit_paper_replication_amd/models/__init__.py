"""Model zoo: ViT (+ blocks), classifier-free ViT backbone, TinyVGG, named presets."""
from .presets import PRESETS, vit, vit_b16, vit_h14, vit_l16
from .tiny_vgg import TinyVGG
from .vit import (MLPBlock, MultiHeadSelfAttentionBlock, PatchEmbedding, SelfAttention, TransformerEncoderBlock,
                  ViT)
from . import vit_no_classifier

__all__ = ["ViT", "PatchEmbedding", "MultiHeadSelfAttentionBlock", "MLPBlock", "TransformerEncoderBlock",
           "SelfAttention", "TinyVGG", "PRESETS", "vit", "vit_b16", "vit_l16", "vit_h14", "vit_no_classifier"]
