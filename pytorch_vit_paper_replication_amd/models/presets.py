"""Named ViT configurations (ViT paper Table 1; reference ctor defaults are ViT-B/16)."""
from __future__ import annotations

from typing import Dict

from .vit import ViT

PRESETS: Dict[str, Dict] = {
    "vit_b16": dict(patch_size=16, num_transformer_layer=12, num_heads=12, embedding_dim=768, mlp_size=3072),
    "vit_b32": dict(patch_size=32, num_transformer_layer=12, num_heads=12, embedding_dim=768, mlp_size=3072),
    "vit_l16": dict(patch_size=16, num_transformer_layer=24, num_heads=16, embedding_dim=1024, mlp_size=4096),
    "vit_l32": dict(patch_size=32, num_transformer_layer=24, num_heads=16, embedding_dim=1024, mlp_size=4096),
    "vit_h14": dict(patch_size=14, num_transformer_layer=32, num_heads=16, embedding_dim=1280, mlp_size=5120),
    "vit_tiny_test": dict(patch_size=8, num_transformer_layer=2, num_heads=2, embedding_dim=128, mlp_size=256),
}


def vit(name: str, image_size: int = 224, num_classes: int = 1000, **overrides) -> ViT:
    cfg = dict(PRESETS[name])
    cfg.update(overrides)
    return ViT(image_size=image_size, num_classes=num_classes, **cfg)


def vit_b16(**kw) -> ViT:
    return vit("vit_b16", **kw)


def vit_l16(**kw) -> ViT:
    return vit("vit_l16", **kw)


def vit_h14(**kw) -> ViT:
    return vit("vit_h14", **kw)
