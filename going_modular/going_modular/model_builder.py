"""Reference-compatible ``model_builder`` (GM/model_builder.py): TinyVGG."""
from pytorch_vit_paper_replication_amd.models.tiny_vgg import TinyVGG  # noqa: F401
