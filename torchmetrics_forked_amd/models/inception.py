"""Inception-v3 feature extractor in the FID ("inception-v3-compat") layout used by FID / KID / IS / MiFID.

Input: uint8 images ``[N, 3, H, W]`` in [0, 255]; resized bilinearly to 299×299, scaled to [-1, 1).  Returns the
requested taps (``'64'``, ``'192'``, ``'768'``, ``'2048'``, ``'logits_unbiased'``, ``'logits'``).  Random init by
default; pass ``weights_path`` to load a compatible state dict (loaded with ``weights_only=True``)."""
from typing import List, Optional, Sequence, Tuple

import torch
import torch.nn.functional as F
from torch import Tensor, nn


class BasicConv2d(nn.Module):
    def __init__(self, c_in: int, c_out: int, **kwargs) -> None:  # noqa: ANN003
        super().__init__()
        self.conv = nn.Conv2d(c_in, c_out, bias=False, **kwargs)
        self.bn = nn.BatchNorm2d(c_out, eps=0.001)

    def forward(self, x: Tensor) -> Tensor:
        return F.relu(self.bn(self.conv(x)), inplace=True)


class InceptionA(nn.Module):
    def __init__(self, c_in: int, pool_features: int) -> None:
        super().__init__()
        self.branch1x1 = BasicConv2d(c_in, 64, kernel_size=1)
        self.branch5x5_1 = BasicConv2d(c_in, 48, kernel_size=1)
        self.branch5x5_2 = BasicConv2d(48, 64, kernel_size=5, padding=2)
        self.branch3x3dbl_1 = BasicConv2d(c_in, 64, kernel_size=1)
        self.branch3x3dbl_2 = BasicConv2d(64, 96, kernel_size=3, padding=1)
        self.branch3x3dbl_3 = BasicConv2d(96, 96, kernel_size=3, padding=1)
        self.branch_pool = BasicConv2d(c_in, pool_features, kernel_size=1)

    def forward(self, x: Tensor) -> Tensor:
        b1 = self.branch1x1(x)
        b5 = self.branch5x5_2(self.branch5x5_1(x))
        b3 = self.branch3x3dbl_3(self.branch3x3dbl_2(self.branch3x3dbl_1(x)))
        bp = self.branch_pool(F.avg_pool2d(x, kernel_size=3, stride=1, padding=1, count_include_pad=False))
        return torch.cat([b1, b5, b3, bp], 1)


class InceptionB(nn.Module):
    def __init__(self, c_in: int) -> None:
        super().__init__()
        self.branch3x3 = BasicConv2d(c_in, 384, kernel_size=3, stride=2)
        self.branch3x3dbl_1 = BasicConv2d(c_in, 64, kernel_size=1)
        self.branch3x3dbl_2 = BasicConv2d(64, 96, kernel_size=3, padding=1)
        self.branch3x3dbl_3 = BasicConv2d(96, 96, kernel_size=3, stride=2)

    def forward(self, x: Tensor) -> Tensor:
        b3 = self.branch3x3(x)
        bd = self.branch3x3dbl_3(self.branch3x3dbl_2(self.branch3x3dbl_1(x)))
        return torch.cat([b3, bd, F.max_pool2d(x, kernel_size=3, stride=2)], 1)


class InceptionC(nn.Module):
    def __init__(self, c_in: int, c7: int) -> None:
        super().__init__()
        self.branch1x1 = BasicConv2d(c_in, 192, kernel_size=1)
        self.branch7x7_1 = BasicConv2d(c_in, c7, kernel_size=1)
        self.branch7x7_2 = BasicConv2d(c7, c7, kernel_size=(1, 7), padding=(0, 3))
        self.branch7x7_3 = BasicConv2d(c7, 192, kernel_size=(7, 1), padding=(3, 0))
        self.branch7x7dbl_1 = BasicConv2d(c_in, c7, kernel_size=1)
        self.branch7x7dbl_2 = BasicConv2d(c7, c7, kernel_size=(7, 1), padding=(3, 0))
        self.branch7x7dbl_3 = BasicConv2d(c7, c7, kernel_size=(1, 7), padding=(0, 3))
        self.branch7x7dbl_4 = BasicConv2d(c7, c7, kernel_size=(7, 1), padding=(3, 0))
        self.branch7x7dbl_5 = BasicConv2d(c7, 192, kernel_size=(1, 7), padding=(0, 3))
        self.branch_pool = BasicConv2d(c_in, 192, kernel_size=1)

    def forward(self, x: Tensor) -> Tensor:
        b1 = self.branch1x1(x)
        b7 = self.branch7x7_3(self.branch7x7_2(self.branch7x7_1(x)))
        bd = x
        for m in (self.branch7x7dbl_1, self.branch7x7dbl_2, self.branch7x7dbl_3, self.branch7x7dbl_4, self.branch7x7dbl_5):
            bd = m(bd)
        bp = self.branch_pool(F.avg_pool2d(x, kernel_size=3, stride=1, padding=1, count_include_pad=False))
        return torch.cat([b1, b7, bd, bp], 1)


class InceptionD(nn.Module):
    def __init__(self, c_in: int) -> None:
        super().__init__()
        self.branch3x3_1 = BasicConv2d(c_in, 192, kernel_size=1)
        self.branch3x3_2 = BasicConv2d(192, 320, kernel_size=3, stride=2)
        self.branch7x7x3_1 = BasicConv2d(c_in, 192, kernel_size=1)
        self.branch7x7x3_2 = BasicConv2d(192, 192, kernel_size=(1, 7), padding=(0, 3))
        self.branch7x7x3_3 = BasicConv2d(192, 192, kernel_size=(7, 1), padding=(3, 0))
        self.branch7x7x3_4 = BasicConv2d(192, 192, kernel_size=3, stride=2)

    def forward(self, x: Tensor) -> Tensor:
        b3 = self.branch3x3_2(self.branch3x3_1(x))
        b7 = self.branch7x7x3_4(self.branch7x7x3_3(self.branch7x7x3_2(self.branch7x7x3_1(x))))
        return torch.cat([b3, b7, F.max_pool2d(x, kernel_size=3, stride=2)], 1)


class InceptionE(nn.Module):
    def __init__(self, c_in: int, pool: str) -> None:
        super().__init__()
        self.pool = pool
        self.branch1x1 = BasicConv2d(c_in, 320, kernel_size=1)
        self.branch3x3_1 = BasicConv2d(c_in, 384, kernel_size=1)
        self.branch3x3_2a = BasicConv2d(384, 384, kernel_size=(1, 3), padding=(0, 1))
        self.branch3x3_2b = BasicConv2d(384, 384, kernel_size=(3, 1), padding=(1, 0))
        self.branch3x3dbl_1 = BasicConv2d(c_in, 448, kernel_size=1)
        self.branch3x3dbl_2 = BasicConv2d(448, 384, kernel_size=3, padding=1)
        self.branch3x3dbl_3a = BasicConv2d(384, 384, kernel_size=(1, 3), padding=(0, 1))
        self.branch3x3dbl_3b = BasicConv2d(384, 384, kernel_size=(3, 1), padding=(1, 0))
        self.branch_pool = BasicConv2d(c_in, 192, kernel_size=1)

    def forward(self, x: Tensor) -> Tensor:
        b1 = self.branch1x1(x)
        b3 = self.branch3x3_1(x)
        b3 = torch.cat([self.branch3x3_2a(b3), self.branch3x3_2b(b3)], 1)
        bd = self.branch3x3dbl_2(self.branch3x3dbl_1(x))
        bd = torch.cat([self.branch3x3dbl_3a(bd), self.branch3x3dbl_3b(bd)], 1)
        if self.pool == "avg":
            bp = F.avg_pool2d(x, kernel_size=3, stride=1, padding=1, count_include_pad=False)
        else:
            bp = F.max_pool2d(x, kernel_size=3, stride=1, padding=1)
        return torch.cat([b1, b3, bd, self.branch_pool(bp)], 1)


class FeatureExtractorInceptionV3(nn.Module):
    INPUT_IMAGE_SIZE = 299
    FEATURES = ("64", "192", "768", "2048", "logits_unbiased", "logits")

    def __init__(self, features_list: Sequence[str] = ("2048",), weights_path: Optional[str] = None, num_classes: int = 1008) -> None:
        super().__init__()
        for f in features_list:
            if f not in self.FEATURES:
                raise ValueError(f"Unknown feature tap {f}; expected one of {self.FEATURES}")
        self.features_list = [str(f) for f in features_list]
        self.Conv2d_1a_3x3 = BasicConv2d(3, 32, kernel_size=3, stride=2)
        self.Conv2d_2a_3x3 = BasicConv2d(32, 32, kernel_size=3)
        self.Conv2d_2b_3x3 = BasicConv2d(32, 64, kernel_size=3, padding=1)
        self.MaxPool_1 = nn.MaxPool2d(kernel_size=3, stride=2)
        self.Conv2d_3b_1x1 = BasicConv2d(64, 80, kernel_size=1)
        self.Conv2d_4a_3x3 = BasicConv2d(80, 192, kernel_size=3)
        self.MaxPool_2 = nn.MaxPool2d(kernel_size=3, stride=2)
        self.Mixed_5b = InceptionA(192, pool_features=32)
        self.Mixed_5c = InceptionA(256, pool_features=64)
        self.Mixed_5d = InceptionA(288, pool_features=64)
        self.Mixed_6a = InceptionB(288)
        self.Mixed_6b = InceptionC(768, c7=128)
        self.Mixed_6c = InceptionC(768, c7=160)
        self.Mixed_6d = InceptionC(768, c7=160)
        self.Mixed_6e = InceptionC(768, c7=192)
        self.Mixed_7a = InceptionD(768)
        self.Mixed_7b = InceptionE(1280, pool="avg")
        self.Mixed_7c = InceptionE(2048, pool="max")
        self.AvgPool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(2048, num_classes)
        if weights_path is not None:
            self.load_state_dict(torch.load(weights_path, map_location="cpu", weights_only=True))
        self.eval()
        for p in self.parameters():
            p.requires_grad_(False)

    def train(self, mode: bool = True) -> "FeatureExtractorInceptionV3":
        return super().train(False)

    def _taps(self, x: Tensor) -> Tuple[Tensor, ...]:
        want = set(self.features_list)
        out = {}
        x = x.float()
        x = F.interpolate(x, size=(self.INPUT_IMAGE_SIZE, self.INPUT_IMAGE_SIZE), mode="bilinear", align_corners=False)
        x = (x - 128) / 128
        x = self.MaxPool_1(self.Conv2d_2b_3x3(self.Conv2d_2a_3x3(self.Conv2d_1a_3x3(x))))
        if "64" in want:
            out["64"] = F.adaptive_avg_pool2d(x, 1).flatten(1)
        x = self.MaxPool_2(self.Conv2d_4a_3x3(self.Conv2d_3b_1x1(x)))
        if "192" in want:
            out["192"] = F.adaptive_avg_pool2d(x, 1).flatten(1)
        for m in (self.Mixed_5b, self.Mixed_5c, self.Mixed_5d, self.Mixed_6a, self.Mixed_6b, self.Mixed_6c, self.Mixed_6d,
                  self.Mixed_6e):
            x = m(x)
        if "768" in want:
            out["768"] = F.adaptive_avg_pool2d(x, 1).flatten(1)
        x = torch.flatten(self.AvgPool(self.Mixed_7c(self.Mixed_7b(self.Mixed_7a(x)))), 1)
        out["2048"] = x
        if "logits_unbiased" in want or "logits" in want:
            lu = x.mm(self.fc.weight.T)
            out["logits_unbiased"] = lu
            out["logits"] = lu + self.fc.bias.unsqueeze(0)
        return tuple(out[f] for f in self.features_list)

    def forward(self, x: Tensor) -> Tensor:
        if x.dtype != torch.uint8:
            raise ValueError("Expecting image as torch.Tensor with dtype=torch.uint8")
        return self._taps(x)[0].reshape(x.shape[0], -1)
