"""torchvision-free image transforms (torchvision is not available on the target image).

Covers what the reference pipelines use (MAIN.ipynb:254-265 v2 ToImage/Resize/ToDtype,
EX.ipynb:225-232 Resize/ToTensor, GM/predictions.py:46-54 Resize/ToTensor/Normalize, and the
pretrained-weights recipe resize-256/center-crop-224/ImageNet-normalise). PIL resampling is
bilinear, like torchvision's default for PIL inputs (antialias on).
"""
from __future__ import annotations

from typing import Sequence, Tuple, Union

import numpy as np
import torch
from PIL import Image

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def _size2(size) -> Tuple[int, int]:
    if isinstance(size, int):
        return size, size
    return int(size[0]), int(size[1])


class Compose:
    def __init__(self, transforms: Sequence):
        self.transforms = list(transforms)

    def __call__(self, x):
        for t in self.transforms:
            x = t(x)
        return x

    def __repr__(self):
        inner = "\n".join(f"    {t!r}" for t in self.transforms)
        return f"Compose(\n{inner}\n)"


class Resize:
    """Resize a PIL image (or CHW tensor). ``size=(h, w)`` is exact; an int resizes the short side."""

    def __init__(self, size: Union[int, Sequence[int]], interpolation=Image.BILINEAR):
        self.size = size
        self.interpolation = interpolation

    def _target(self, w: int, h: int) -> Tuple[int, int]:
        if isinstance(self.size, int):
            s = self.size
            if w <= h:
                return s, int(round(s * h / w))
            return int(round(s * w / h)), s
        hh, ww = _size2(self.size)
        return ww, hh

    def __call__(self, img):
        if isinstance(img, torch.Tensor):
            h, w = img.shape[-2:]
            tw, th = self._target(w, h)
            x = img.unsqueeze(0) if img.dim() == 3 else img
            out = torch.nn.functional.interpolate(x.float(), size=(th, tw), mode="bilinear", align_corners=False,
                                                  antialias=True)
            if img.dtype == torch.uint8:  # like torchvision: integer images stay integer
                out = out.round_().clamp_(0, 255).to(torch.uint8)
            return out.squeeze(0) if img.dim() == 3 else out
        tw, th = self._target(*img.size)
        return img.resize((tw, th), self.interpolation)

    def __repr__(self):
        return f"Resize(size={self.size}, interpolation=bilinear)"


class CenterCrop:
    def __init__(self, size):
        self.size = _size2(size)

    def __call__(self, img):
        th, tw = self.size
        if isinstance(img, torch.Tensor):
            h, w = img.shape[-2:]
            top, left = int(round((h - th) / 2.0)), int(round((w - tw) / 2.0))
            return img[..., top:top + th, left:left + tw]
        w, h = img.size
        left, top = int(round((w - tw) / 2.0)), int(round((h - th) / 2.0))
        return img.crop((left, top, left + tw, top + th))

    def __repr__(self):
        return f"CenterCrop(size={self.size})"


def _pil_to_uint8_chw(img) -> torch.Tensor:
    if not isinstance(img, Image.Image):
        raise TypeError(f"expected a PIL image, got {type(img)}")
    img = img.convert("RGB") if img.mode not in ("RGB", "L") else img
    a = np.asarray(img, dtype=np.uint8)
    if a.ndim == 2:
        a = a[:, :, None]
    return torch.from_numpy(a.copy()).permute(2, 0, 1).contiguous()


class ToTensor:
    """PIL [H,W,C] uint8 -> float32 CHW in [0, 1]."""

    def __call__(self, img):
        if isinstance(img, torch.Tensor):
            return img.float() / 255.0 if img.dtype == torch.uint8 else img
        return _pil_to_uint8_chw(img).float().div_(255.0)

    def __repr__(self):
        return "ToTensor()"


class ToImage:
    """v2.ToImage: PIL -> uint8 CHW tensor."""

    def __call__(self, img):
        return img if isinstance(img, torch.Tensor) else _pil_to_uint8_chw(img)

    def __repr__(self):
        return "ToImage()"


class ToDtype:
    """v2.ToDtype(dtype, scale=True): uint8 [0,255] -> float [0,1] when scale."""

    def __init__(self, dtype=torch.float32, scale: bool = False):
        self.dtype, self.scale = dtype, scale

    def __call__(self, x: torch.Tensor):
        if self.scale and x.dtype == torch.uint8 and self.dtype.is_floating_point:
            return x.to(self.dtype).div_(255.0)
        return x.to(self.dtype)

    def __repr__(self):
        return f"ToDtype(dtype={self.dtype}, scale={self.scale})"


class Normalize:
    def __init__(self, mean=IMAGENET_MEAN, std=IMAGENET_STD):
        self.mean = torch.tensor(mean, dtype=torch.float32).view(-1, 1, 1)
        self.std = torch.tensor(std, dtype=torch.float32).view(-1, 1, 1)

    def __call__(self, x: torch.Tensor):
        return (x - self.mean.to(x.device)) / self.std.to(x.device)

    def __repr__(self):
        return f"Normalize(mean={self.mean.flatten().tolist()}, std={self.std.flatten().tolist()})"


def default_vit_transform(image_size: int = 224) -> Compose:
    """The reference's manual transform (MAIN.ipynb:254-265): Resize -> [0,1] float, no normalisation."""
    return Compose([ToImage(), Resize((image_size, image_size)), ToDtype(torch.float32, scale=True)])


def imagenet_eval_transform(image_size: int = 224, resize: int = 256) -> Compose:
    """The pretrained-weights recipe: resize short side, center crop, ImageNet normalisation."""
    return Compose([Resize(resize), CenterCrop(image_size), ToTensor(), Normalize()])


class v2:  # namespace mirroring torchvision.transforms.v2 names used by the reference
    Compose = Compose
    Resize = Resize
    CenterCrop = CenterCrop
    ToImage = ToImage
    ToDtype = ToDtype
    Normalize = Normalize
