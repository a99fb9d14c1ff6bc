"""Utilities: checkpointing (reference GM/utils.py), seeding, metrics, summaries, plots, profiling."""
from .checkpoint import load_checkpoint, load_model, portable_state_dict, save_checkpoint, save_model
from .seed import set_all_seeds, set_seeds
from .summary import count_params, summary

__all__ = ["save_model", "load_model", "save_checkpoint", "load_checkpoint", "portable_state_dict", "set_seeds",
           "set_all_seeds", "summary", "count_params"]
