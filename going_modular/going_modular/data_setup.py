"""Reference-compatible ``data_setup`` (GM/data_setup.py): create_dataloaders, NUM_WORKERS."""
from pytorch_vit_paper_replication_amd.data.loaders import NUM_WORKERS, create_dataloaders  # noqa: F401
