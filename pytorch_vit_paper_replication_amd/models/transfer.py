"""Transfer learning: torchvision-format ViT checkpoints and the frozen-backbone feature extractor.

The reference's transfer-learning section loads torchvision's pretrained
``vit_b_16`` (MAIN.ipynb:4036-4041), freezes every parameter (MAIN.ipynb:4111-4113), swaps the head for
``Linear(768, n_classes)`` (MAIN.ipynb:4128-4130) and trains with ``engine.train``. torchvision is not
part of this stack and there is no network, so the equivalent here is:

  * ``from_torchvision_state_dict``: rename a torchvision ``VisionTransformer`` state_dict (a local
    file, loaded with ``torch.load(weights_only=True)``) to this framework's ViT keys, so the
    pretrained weights run on the fused MI355X path; ``to_torchvision_state_dict`` is the inverse;
  * ``vit_from_torchvision_checkpoint``: build the matching ``ViT`` (LayerNorm eps 1e-6, as
    torchvision uses) and load the converted weights;
  * ``feature_extractor``: freeze the backbone and install a fresh classifier head.

The key mapping covers both torchvision MLP naming schemes (``mlp.0`` / ``mlp.3`` and the older
``mlp.linear_1`` / ``mlp.linear_2``). Parity against real torchvision weights is unpinned (no
torchvision / checkpoint in this environment); tests pin the mapping with synthetic state dicts.
"""
from __future__ import annotations

import re
from typing import Dict, Optional

import torch
from torch import nn

from .vit import ViT

_LAYER_RE = re.compile(r"^encoder\.layers\.encoder_layer_(\d+)\.(.+)$")

# torchvision encoder-layer suffix -> this framework's block suffix
_TV_TO_OURS = {
    "ln_1.weight": "msa_block.layer_norm.weight",
    "ln_1.bias": "msa_block.layer_norm.bias",
    "self_attention.in_proj_weight": "msa_block.multi_head_attention.in_proj_weight",
    "self_attention.in_proj_bias": "msa_block.multi_head_attention.in_proj_bias",
    "self_attention.out_proj.weight": "msa_block.multi_head_attention.out_proj.weight",
    "self_attention.out_proj.bias": "msa_block.multi_head_attention.out_proj.bias",
    "ln_2.weight": "mlp_block.layer_norm.weight",
    "ln_2.bias": "mlp_block.layer_norm.bias",
    "mlp.0.weight": "mlp_block.mlp.0.weight",
    "mlp.0.bias": "mlp_block.mlp.0.bias",
    "mlp.3.weight": "mlp_block.mlp.3.weight",
    "mlp.3.bias": "mlp_block.mlp.3.bias",
    "mlp.linear_1.weight": "mlp_block.mlp.0.weight",
    "mlp.linear_1.bias": "mlp_block.mlp.0.bias",
    "mlp.linear_2.weight": "mlp_block.mlp.3.weight",
    "mlp.linear_2.bias": "mlp_block.mlp.3.bias",
}
_TOP_TV_TO_OURS = {
    "class_token": "patch_embedding_block.class_token",
    "conv_proj.weight": "patch_embedding_block.patch_and_flatten.0.weight",
    "conv_proj.bias": "patch_embedding_block.patch_and_flatten.0.bias",
    "encoder.pos_embedding": "patch_embedding_block.position_embedding",
    "encoder.ln.weight": "layer_norm.weight",
    "encoder.ln.bias": "layer_norm.bias",
    "heads.head.weight": "classifier.0.weight",
    "heads.head.bias": "classifier.0.bias",
}
TORCHVISION_LN_EPS = 1e-6


def from_torchvision_state_dict(sd: Dict[str, torch.Tensor], drop_head: bool = False) -> Dict[str, torch.Tensor]:
    """torchvision ``VisionTransformer`` keys -> this framework's ``ViT`` keys (tensors shared)."""
    out: Dict[str, torch.Tensor] = {}
    for k, v in sd.items():
        if k in _TOP_TV_TO_OURS:
            nk = _TOP_TV_TO_OURS[k]
            if drop_head and nk.startswith("classifier."):
                continue
            out[nk] = v
            continue
        m = _LAYER_RE.match(k)
        if m and m.group(2) in _TV_TO_OURS:
            out[f"transformer_encoder.{m.group(1)}.{_TV_TO_OURS[m.group(2)]}"] = v
            continue
        if k.startswith("heads.pre_logits"):
            raise ValueError("torchvision ViTs with a representation (pre_logits) layer have no equivalent here")
        raise KeyError(f"unrecognised torchvision ViT key: {k}")
    return out


def to_torchvision_state_dict(sd: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    """Inverse of ``from_torchvision_state_dict`` (uses torchvision >= 0.15 ``mlp.0`` / ``mlp.3`` names)."""
    top = {v: k for k, v in _TOP_TV_TO_OURS.items()}
    blk = {v: k for k, v in _TV_TO_OURS.items() if "linear_" not in k}
    out: Dict[str, torch.Tensor] = {}
    for k, v in sd.items():
        if k in top:
            out[top[k]] = v
            continue
        m = re.match(r"^transformer_encoder\.(\d+)\.(.+)$", k)
        if m and m.group(2) in blk:
            out[f"encoder.layers.encoder_layer_{m.group(1)}.{blk[m.group(2)]}"] = v
            continue
        raise KeyError(f"unrecognised ViT key: {k}")
    return out


def _infer_config(sd: Dict[str, torch.Tensor]) -> dict:
    w = sd["conv_proj.weight"]
    D, _, P, _ = w.shape
    n_tok = sd["encoder.pos_embedding"].shape[1]
    side = int(round((n_tok - 1) ** 0.5))
    layers = 1 + max(int(m.group(1)) for m in map(_LAYER_RE.match, sd) if m)
    mlp = next(v.shape[0] for k, v in sd.items() if k.endswith(("mlp.0.weight", "mlp.linear_1.weight")))
    return dict(image_size=side * P, patch_size=P, num_transformer_layer=layers, embedding_dim=D, mlp_size=mlp)


def set_layernorm_eps(model: nn.Module, eps: float) -> nn.Module:
    for m in model.modules():
        if isinstance(m, nn.LayerNorm):
            m.eps = eps
    return model


def vit_from_torchvision_checkpoint(path: str, num_heads: Optional[int] = None, num_classes: Optional[int] = None,
                                    **overrides) -> ViT:
    """Build a ViT from a local torchvision checkpoint file (loaded with ``weights_only=True``)."""
    sd = torch.load(path, map_location="cpu", weights_only=True)
    if "state_dict" in sd and isinstance(sd["state_dict"], dict):
        sd = sd["state_dict"]
    cfg = _infer_config(sd)
    cfg["num_heads"] = num_heads or max(1, cfg["embedding_dim"] // 64)
    head_classes = sd["heads.head.weight"].shape[0] if "heads.head.weight" in sd else None
    cfg["num_classes"] = num_classes or head_classes or 1000
    cfg.update(overrides)
    model = set_layernorm_eps(ViT(**cfg), TORCHVISION_LN_EPS)
    keep_head = head_classes is not None and head_classes == cfg["num_classes"]
    ours = from_torchvision_state_dict(sd, drop_head=not keep_head)
    missing, unexpected = model.load_state_dict(ours, strict=False)
    allowed_missing = set() if keep_head else {"classifier.0.weight", "classifier.0.bias"}
    if set(missing) - allowed_missing or unexpected:
        raise RuntimeError(f"checkpoint mismatch: missing {missing}, unexpected {unexpected}")
    return model


def feature_extractor(model: ViT, num_classes: int, freeze: bool = True, seed: Optional[int] = None) -> ViT:
    """Freeze the backbone and install a fresh ``Linear(D, num_classes)`` head (MAIN.ipynb:4111-4130).

    Only the new head is trainable; the fused path skips every frozen weight gradient (their GEMMs
    are not launched), so fine-tuning costs one forward plus the head's backward per step."""
    if freeze:
        for p in model.parameters():
            p.requires_grad = False
    if seed is not None:
        torch.manual_seed(seed)
    D = model.classifier[0].in_features if isinstance(model.classifier, nn.Sequential) else model.config["embedding_dim"]
    dev = next(model.parameters()).device
    model.classifier = nn.Sequential(nn.Linear(in_features=D, out_features=num_classes)).to(dev)
    model.config["num_classes"] = num_classes
    return model
