"""Image gradients (API parity: reference ``functional/image/gradients.py:20-80``)."""
from typing import Tuple

import torch
import torch.nn.functional as F
from torch import Tensor


def _image_gradients_validate(img: Tensor) -> None:
    if not isinstance(img, Tensor):
        raise TypeError(f"The `img` expects a value of <Tensor> type but got {type(img)}")
    if img.ndim != 4:
        raise RuntimeError(f"The `img` expects a 4D tensor but got {img.ndim}D tensor")


def _compute_image_gradients(img: Tensor) -> Tuple[Tensor, Tensor]:
    dy = F.pad(img[..., 1:, :] - img[..., :-1, :], (0, 0, 0, 1))
    dx = F.pad(img[..., :, 1:] - img[..., :, :-1], (0, 1, 0, 0))
    return dy, dx


def image_gradients(img: Tensor) -> Tuple[Tensor, Tensor]:
    _image_gradients_validate(img)
    return _compute_image_gradients(img)
