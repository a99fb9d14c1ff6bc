"""Compatibility module for ``models/vit_no_classifier.py`` of the reference."""
from pytorch_vit_paper_replication_amd.models.vit_no_classifier import (MLPBlock,  # noqa: F401
                                                                        MultiHeadSelfAttentionBlock, PatchEmbedding,
                                                                        TransformerEncoderBlock, ViT)
