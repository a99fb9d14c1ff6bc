"""Reference-compatible ``utils`` (GM/utils.py): save_model (+ load_model, checkpoints)."""
from pytorch_vit_paper_replication_amd.utils.checkpoint import (load_checkpoint, load_model,  # noqa: F401
                                                                save_checkpoint, save_model)
