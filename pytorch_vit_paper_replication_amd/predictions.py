"""Single-image prediction (reference GM/predictions.py:20-83) without torchvision."""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch
from PIL import Image

from .data import transforms as T

device = "cuda" if torch.cuda.is_available() else "cpu"


def predict_image(model: torch.nn.Module, image_path: str, image_size: Tuple[int, int] = (224, 224),
                  transform=None, device: torch.device = device) -> Tuple[int, torch.Tensor, Image.Image]:
    img = Image.open(image_path)
    image_transform = transform if transform is not None else T.Compose(
        [T.Resize(image_size), T.ToTensor(), T.Normalize(mean=[0.485, 0.456, 0.406], std=[0.229, 0.224, 0.225])])
    model.to(device)
    model.eval()
    with torch.inference_mode():
        transformed_image = image_transform(img.convert("RGB")).unsqueeze(dim=0)
        logits = model(transformed_image.to(device))
    probs = torch.softmax(logits.float(), dim=1)
    label = int(torch.argmax(probs, dim=1))
    return label, probs.cpu(), img


def pred_and_plot_image(model: torch.nn.Module, class_names: List[str], image_path: str,
                        image_size: Tuple[int, int] = (224, 224), transform=None, device: torch.device = device,
                        save_path: Optional[str] = None):
    """Predict and plot ``Pred: <class> | Prob: <p>`` like the reference; returns None."""
    label, probs, img = predict_image(model, image_path, image_size, transform, device)
    import matplotlib

    if save_path:
        matplotlib.use("Agg")
    import matplotlib.pyplot as plt

    plt.figure()
    plt.imshow(img)
    plt.title(f"Pred: {class_names[label]} | Prob: {probs.max():.3f}")
    plt.axis(False)
    if save_path:
        plt.savefig(save_path)
        plt.close()
