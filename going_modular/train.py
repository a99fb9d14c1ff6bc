"""Reference-compatible script trainer (GM/train.py), fixed: it passes the required LR scheduler
(the reference call omitted it and raised TypeError) and can train a ViT on synthetic data.
Run ``python -m pytorch_vit_paper_replication_amd.cli.train --help`` for all options."""
import sys

from pytorch_vit_paper_replication_amd.cli.train import main

if __name__ == "__main__":
    sys.exit(main())
