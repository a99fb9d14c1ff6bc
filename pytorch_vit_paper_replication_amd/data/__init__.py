"""Data pipeline: torchvision-free ImageFolder + transforms, synthetic ImageNet-shaped sources,
and ``create_dataloaders`` with the reference signature (GM/data_setup.py:12-65)."""
from .image_folder import IMG_EXTENSIONS, ImageFolder, pil_loader
from .loaders import NUM_WORKERS, create_dataloaders, create_synthetic_dataloaders
from .prefetch import DevicePrefetcher, prefetch
from .synthetic import DeviceSyntheticLoader, SyntheticImageNet
from . import transforms

__all__ = ["ImageFolder", "pil_loader", "IMG_EXTENSIONS", "create_dataloaders", "create_synthetic_dataloaders",
           "NUM_WORKERS", "SyntheticImageNet", "DeviceSyntheticLoader", "DevicePrefetcher", "prefetch", "transforms"]
