"""Model zoo: ViT (+ blocks), classifier-free ViT backbone, TinyVGG, named presets."""
from .presets import PRESETS, vit, vit_b16, vit_h14, vit_l16
from .tiny_vgg import TinyVGG
from .vit import (MLPBlock, MultiHeadSelfAttentionBlock, PatchEmbedding, SelfAttention, TransformerEncoderBlock,
                  ViT)
from . import vit_no_classifier
from .notebook import PatchEmbeddingV1
from .transfer import (feature_extractor, from_torchvision_state_dict, to_torchvision_state_dict,
                       vit_from_torchvision_checkpoint)
from .vit_torch_encoder import ViTTorchEncoder

__all__ = ["ViT", "PatchEmbedding", "MultiHeadSelfAttentionBlock", "MLPBlock", "TransformerEncoderBlock",
           "SelfAttention", "TinyVGG", "PRESETS", "vit", "vit_b16", "vit_l16", "vit_h14", "vit_no_classifier",
           "PatchEmbeddingV1", "ViTTorchEncoder", "feature_extractor", "from_torchvision_state_dict",
           "to_torchvision_state_dict", "vit_from_torchvision_checkpoint"]
