"""Reference-compatible import path: ``from models.vit import ViT`` (reference models/vit.py)."""
