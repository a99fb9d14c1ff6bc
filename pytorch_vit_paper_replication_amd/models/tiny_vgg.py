"""TinyVGG (reference GM/model_builder.py:7-56): the CNN-explainer model used by the script trainer."""
import torch
from torch import nn


class TinyVGG(nn.Module):
    """2x(Conv3x3-ReLU-Conv3x3-ReLU-MaxPool2) -> Flatten -> Linear(hidden*13*13, out); 64x64 inputs."""

    def __init__(self, input_shape: int, hidden_units: int, output_shape: int) -> None:
        super().__init__()
        self.conv_block_1 = nn.Sequential(
            nn.Conv2d(input_shape, hidden_units, kernel_size=3, stride=1, padding=0), nn.ReLU(),
            nn.Conv2d(hidden_units, hidden_units, kernel_size=3, stride=1, padding=0), nn.ReLU(),
            nn.MaxPool2d(kernel_size=2, stride=2))
        self.conv_block_2 = nn.Sequential(
            nn.Conv2d(hidden_units, hidden_units, kernel_size=3, padding=0), nn.ReLU(),
            nn.Conv2d(hidden_units, hidden_units, kernel_size=3, padding=0), nn.ReLU(),
            nn.MaxPool2d(2))
        self.classifier = nn.Sequential(nn.Flatten(), nn.Linear(in_features=hidden_units * 13 * 13,
                                                                out_features=output_shape))

    def forward(self, x: torch.Tensor):
        return self.classifier(self.conv_block_2(self.conv_block_1(x)))
