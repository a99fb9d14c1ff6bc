"""pytorch_vit_paper_replication_amd — an MI355X-native (gfx950 / CDNA4) Vision Transformer
training framework with the public surface of AvalonEnjoyer/pytorch-ViT-paper-replication.

Layers: ``csrc`` HIP kernels -> ``ops`` autograd Functions -> ``models`` ->
``engine`` / ``data`` / ``optim`` / ``parallel`` (RCCL DP) / ``runtime`` (param store, graphs) /
``utils`` (checkpointing, profiling).
"""
__version__ = "0.1.0"

from . import _ext
from .models import MLPBlock, MultiHeadSelfAttentionBlock, PatchEmbedding, TinyVGG, TransformerEncoderBlock, ViT

__all__ = ["ViT", "PatchEmbedding", "MultiHeadSelfAttentionBlock", "MLPBlock", "TransformerEncoderBlock", "TinyVGG",
           "_ext", "__version__"]
