"""Reference-compatible ``engine`` (GM/engine.py): train / train_step / test_step."""
from pytorch_vit_paper_replication_amd.engine import test_step, train, train_step  # noqa: F401
