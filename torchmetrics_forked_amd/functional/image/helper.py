"""Image window helpers (behavioural parity: reference ``functional/image/helper.py``)."""
from typing import Sequence, Tuple, Union

import torch
import torch.nn.functional as F
from torch import Tensor


def _gaussian(kernel_size: int, sigma: float, dtype: torch.dtype, device: Union[torch.device, str]) -> Tensor:
    """Normalised 1-D Gaussian ``[1, kernel_size]``."""
    dist = torch.arange(start=(1 - kernel_size) / 2, end=(1 + kernel_size) / 2, step=1, dtype=dtype, device=device)
    gauss = torch.exp(-((dist / sigma) ** 2) / 2)
    return (gauss / gauss.sum()).unsqueeze(dim=0)


def _gaussian_kernel_2d(
    channel: int, kernel_size: Sequence[int], sigma: Sequence[float], dtype: torch.dtype, device: Union[torch.device, str]
) -> Tensor:
    gx = _gaussian(kernel_size[0], sigma[0], dtype, device)
    gy = _gaussian(kernel_size[1], sigma[1], dtype, device)
    return torch.matmul(gx.t(), gy).expand(channel, 1, kernel_size[0], kernel_size[1])


def _gaussian_kernel_3d(
    channel: int, kernel_size: Sequence[int], sigma: Sequence[float], dtype: torch.dtype, device: torch.device
) -> Tensor:
    gx = _gaussian(kernel_size[0], sigma[0], dtype, device)
    gy = _gaussian(kernel_size[1], sigma[1], dtype, device)
    gz = _gaussian(kernel_size[2], sigma[2], dtype, device)
    kxy = torch.matmul(gx.t(), gy)
    kernel = kxy.unsqueeze(-1) * gz.reshape(1, 1, -1)
    return kernel.expand(channel, 1, *kernel_size)


def _uniform_weight_bias_conv2d(inputs: Tensor, window_size: int) -> Tuple[Tensor, Tensor]:
    weight = torch.full((1, 1, window_size, window_size), 1.0 / window_size**2, dtype=inputs.dtype, device=inputs.device)
    return weight, torch.zeros(1, dtype=inputs.dtype, device=inputs.device)


def _single_dimension_pad(inputs: Tensor, dim: int, pad: int, outer_pad: int = 0) -> Tensor:
    """Symmetric (edge-including) reflection used by the reference's uniform filter."""
    size = inputs.shape[dim]
    front = torch.index_select(inputs, dim, torch.arange(pad - 1, -1, -1, device=inputs.device))
    back = torch.index_select(inputs, dim, torch.arange(size - 1, size - pad - outer_pad, -1, device=inputs.device))
    return torch.cat((front, inputs, back), dim)


def _reflection_pad_2d(inputs: Tensor, pad: int, outer_pad: int = 0) -> Tensor:
    for dim in (2, 3):
        inputs = _single_dimension_pad(inputs, dim, pad, outer_pad)
    return inputs


def _uniform_filter(inputs: Tensor, window_size: int) -> Tensor:
    """Per-channel box filter (all channels in one grouped conv instead of a Python loop over channels)."""
    inputs = _reflection_pad_2d(inputs, window_size // 2, window_size % 2)
    weight, _ = _uniform_weight_bias_conv2d(inputs, window_size)
    c = inputs.shape[1]
    return F.conv2d(inputs, weight.expand(c, 1, window_size, window_size), groups=c)


def _reflection_pad_3d(inputs: Tensor, pad_h: int, pad_w: int, pad_d: int) -> Tensor:
    return F.pad(inputs, (pad_h, pad_h, pad_w, pad_w, pad_d, pad_d), mode="reflect")
