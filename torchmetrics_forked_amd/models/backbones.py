"""Convolutional backbones for LPIPS (layer indices identical to torchvision's ``.features`` so the reference's
slicing ``[0:2], [2:5], ...`` and torchvision checkpoints apply unchanged)."""
from typing import List

import torch
from torch import nn


def alexnet_features() -> nn.Sequential:
    return nn.Sequential(
        nn.Conv2d(3, 64, kernel_size=11, stride=4, padding=2), nn.ReLU(inplace=True),
        nn.MaxPool2d(kernel_size=3, stride=2),
        nn.Conv2d(64, 192, kernel_size=5, padding=2), nn.ReLU(inplace=True),
        nn.MaxPool2d(kernel_size=3, stride=2),
        nn.Conv2d(192, 384, kernel_size=3, padding=1), nn.ReLU(inplace=True),
        nn.Conv2d(384, 256, kernel_size=3, padding=1), nn.ReLU(inplace=True),
        nn.Conv2d(256, 256, kernel_size=3, padding=1), nn.ReLU(inplace=True),
        nn.MaxPool2d(kernel_size=3, stride=2),
    )


def vgg16_features() -> nn.Sequential:
    cfg: List = [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"]
    layers: List[nn.Module] = []
    c_in = 3
    for v in cfg:
        if v == "M":
            layers.append(nn.MaxPool2d(kernel_size=2, stride=2))
        else:
            layers += [nn.Conv2d(c_in, v, kernel_size=3, padding=1), nn.ReLU(inplace=True)]
            c_in = v
    return nn.Sequential(*layers)


class Fire(nn.Module):
    def __init__(self, inplanes: int, squeeze: int, expand1x1: int, expand3x3: int) -> None:
        super().__init__()
        self.squeeze = nn.Conv2d(inplanes, squeeze, kernel_size=1)
        self.squeeze_activation = nn.ReLU(inplace=True)
        self.expand1x1 = nn.Conv2d(squeeze, expand1x1, kernel_size=1)
        self.expand1x1_activation = nn.ReLU(inplace=True)
        self.expand3x3 = nn.Conv2d(squeeze, expand3x3, kernel_size=3, padding=1)
        self.expand3x3_activation = nn.ReLU(inplace=True)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = self.squeeze_activation(self.squeeze(x))
        return torch.cat([self.expand1x1_activation(self.expand1x1(x)), self.expand3x3_activation(self.expand3x3(x))], 1)


def squeezenet1_1_features() -> nn.Sequential:
    return nn.Sequential(
        nn.Conv2d(3, 64, kernel_size=3, stride=2), nn.ReLU(inplace=True),
        nn.MaxPool2d(kernel_size=3, stride=2, ceil_mode=True),
        Fire(64, 16, 64, 64), Fire(128, 16, 64, 64),
        nn.MaxPool2d(kernel_size=3, stride=2, ceil_mode=True),
        Fire(128, 32, 128, 128), Fire(256, 32, 128, 128),
        nn.MaxPool2d(kernel_size=3, stride=2, ceil_mode=True),
        Fire(256, 48, 192, 192), Fire(384, 48, 192, 192), Fire(384, 64, 256, 256), Fire(512, 64, 256, 256),
    )
