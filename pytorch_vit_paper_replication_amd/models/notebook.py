"""Teaching-scaffold modules from the reference notebook.

``PatchEmbeddingV1`` is the first patch embedding of MAIN.ipynb:1382-1419: Conv2d(k=P, s=P) +
Flatten, returning ``[B, N, D]`` patch embeddings only (no class token, no position embedding) and
asserting in ``forward`` that the input resolution is divisible by the patch size (MAIN.ipynb:1413).
The notebook's v2 (MAIN.ipynb:1761-1823) is ``models.PatchEmbedding`` with its global-variable bug
fixed, exactly as the reference's ``models/vit.py:40`` fixes it.
"""
from __future__ import annotations

import torch
from torch import nn


class PatchEmbeddingV1(nn.Module):
    def __init__(self, in_channels: int = 3, patch_size: int = 16, embedding_dim: int = 768):
        super().__init__()
        self.patch_size = patch_size
        self.patcher = nn.Conv2d(in_channels=in_channels, out_channels=embedding_dim, kernel_size=patch_size,
                                 stride=patch_size, padding=0)
        self.flatten = nn.Flatten(start_dim=2, end_dim=3)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        image_resolution = x.shape[-1]
        assert image_resolution % self.patch_size == 0, (
            f"Input image size must be divisble by patch size, image shape: {image_resolution}, "
            f"patch size: {self.patch_size}")
        return self.flatten(self.patcher(x)).permute(0, 2, 1)
