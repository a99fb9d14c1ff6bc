"""ImageFolder without torchvision: ``root/<class>/<image>``, classes sorted by name
(same contract as ``torchvision.datasets.ImageFolder`` used at reference GM/data_setup.py:43-47)."""
from __future__ import annotations

import os
from pathlib import Path
from typing import Callable, List, Optional, Tuple

from PIL import Image
from torch.utils.data import Dataset

IMG_EXTENSIONS = (".jpg", ".jpeg", ".png", ".ppm", ".bmp", ".pgm", ".tif", ".tiff", ".webp")


def pil_loader(path: str) -> Image.Image:
    with open(path, "rb") as f:
        img = Image.open(f)
        return img.convert("RGB")


class ImageFolder(Dataset):
    def __init__(self, root: str, transform: Optional[Callable] = None, target_transform: Optional[Callable] = None,
                 loader: Callable[[str], object] = pil_loader, extensions=IMG_EXTENSIONS):
        self.root = str(root)
        self.transform = transform
        self.target_transform = target_transform
        self.loader = loader
        classes = sorted(e.name for e in os.scandir(self.root) if e.is_dir())
        if not classes:
            raise FileNotFoundError(f"Couldn't find any class folder in {self.root}.")
        self.classes: List[str] = classes
        self.class_to_idx = {c: i for i, c in enumerate(classes)}
        samples: List[Tuple[str, int]] = []
        for c in classes:
            for dirpath, _, files in sorted(os.walk(Path(self.root) / c, followlinks=True)):
                for fn in sorted(files):
                    if fn.lower().endswith(tuple(extensions)):
                        samples.append((os.path.join(dirpath, fn), self.class_to_idx[c]))
        if not samples:
            raise FileNotFoundError(f"Found no valid image file in {self.root}")
        self.samples = samples
        self.imgs = samples
        self.targets = [s[1] for s in samples]

    def __len__(self) -> int:
        return len(self.samples)

    def __getitem__(self, index: int):
        path, target = self.samples[index]
        img = self.loader(path)
        if self.transform is not None:
            img = self.transform(img)
        if self.target_transform is not None:
            target = self.target_transform(target)
        return img, target
