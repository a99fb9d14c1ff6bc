"""Compatibility module for ``models/vit.py`` of the reference (same classes, same signatures)."""
from pytorch_vit_paper_replication_amd.models.vit import (MLPBlock, MultiHeadSelfAttentionBlock,  # noqa: F401
                                                          PatchEmbedding, SelfAttention, TransformerEncoderBlock, ViT)
