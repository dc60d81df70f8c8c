"""Universal image quality index (API parity: reference ``functional/image/uqi.py:23-150``)."""
from typing import Optional, Sequence, Tuple

import torch
import torch.nn.functional as F
from torch import Tensor
from typing_extensions import Literal

from torchmetrics_forked_amd.functional.image.helper import _gaussian_kernel_2d
from torchmetrics_forked_amd.utilities.checks import _check_same_shape
from torchmetrics_forked_amd.utilities.distributed import reduce


def _uqi_update(preds: Tensor, target: Tensor) -> Tuple[Tensor, Tensor]:
    if preds.dtype != target.dtype:
        raise TypeError(
            "Expected `preds` and `target` to have the same data type."
            f" Got preds: {preds.dtype} and target: {target.dtype}."
        )
    _check_same_shape(preds, target)
    if len(preds.shape) != 4:
        raise ValueError(
            f"Expected `preds` and `target` to have BxCxHxW shape. Got preds: {preds.shape} and target: {target.shape}."
        )
    return preds, target


def _uqi_compute(
    preds: Tensor,
    target: Tensor,
    kernel_size: Sequence[int] = (11, 11),
    sigma: Sequence[float] = (1.5, 1.5),
    reduction: Optional[Literal["elementwise_mean", "sum", "none"]] = "elementwise_mean",
) -> Tensor:
    if len(kernel_size) != 2 or len(sigma) != 2:
        raise ValueError(
            "Expected `kernel_size` and `sigma` to have the length of two."
            f" Got kernel_size: {len(kernel_size)} and sigma: {len(sigma)}."
        )
    if any(x % 2 == 0 or x <= 0 for x in kernel_size):
        raise ValueError(f"Expected `kernel_size` to have odd positive number. Got {kernel_size}.")
    if any(y <= 0 for y in sigma):
        raise ValueError(f"Expected `sigma` to have positive number. Got {sigma}.")
    channel, dtype, device = preds.size(1), preds.dtype, preds.device
    kernel = _gaussian_kernel_2d(channel, kernel_size, sigma, dtype, device)
    pad_h, pad_w = (kernel_size[0] - 1) // 2, (kernel_size[1] - 1) // 2
    preds = F.pad(preds, (pad_h, pad_h, pad_w, pad_w), mode="reflect")
    target = F.pad(target, (pad_h, pad_h, pad_w, pad_w), mode="reflect")
    out = F.conv2d(torch.cat((preds, target, preds * preds, target * target, preds * target)), kernel, groups=channel)
    mu_p, mu_t, e_pp, e_tt, e_pt = out.split(preds.shape[0])
    mu_pp, mu_tt, mu_pt = mu_p.pow(2), mu_t.pow(2), mu_p * mu_t
    s_pp, s_tt, s_pt = e_pp - mu_pp, e_tt - mu_tt, e_pt - mu_pt
    upper = 2 * s_pt
    lower = s_pp + s_tt + torch.finfo(s_pp.dtype).eps
    uqi_idx = 2 * mu_pt * upper / ((mu_pp + mu_tt) * lower)
    return reduce(uqi_idx[..., pad_h:-pad_h, pad_w:-pad_w], reduction)


def universal_image_quality_index(
    preds: Tensor,
    target: Tensor,
    kernel_size: Sequence[int] = (11, 11),
    sigma: Sequence[float] = (1.5, 1.5),
    reduction: Optional[Literal["elementwise_mean", "sum", "none"]] = "elementwise_mean",
) -> Tensor:
    preds, target = _uqi_update(preds, target)
    return _uqi_compute(preds, target, kernel_size, sigma, reduction)
