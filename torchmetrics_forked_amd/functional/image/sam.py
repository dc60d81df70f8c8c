"""Spectral angle mapper (API parity: reference ``functional/image/sam.py:22-100``)."""
from typing import Tuple

import torch
from torch import Tensor
from typing_extensions import Literal

from torchmetrics_forked_amd.utilities.checks import _check_same_shape
from torchmetrics_forked_amd.utilities.distributed import reduce


def _sam_update(preds: Tensor, target: Tensor) -> Tuple[Tensor, Tensor]:
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
    if preds.shape[1] <= 1 or target.shape[1] <= 1:
        raise ValueError(
            "Expected channel dimension of `preds` and `target` to be larger than 1."
            f" Got preds: {preds.shape[1]} and target: {target.shape[1]}."
        )
    return preds, target


def _sam_compute(preds: Tensor, target: Tensor, reduction: Literal["elementwise_mean", "sum", "none", None] = "elementwise_mean") -> Tensor:
    dot = (preds * target).sum(dim=1)
    score = torch.clamp(dot / (preds.norm(dim=1) * target.norm(dim=1)), -1, 1).acos()
    return reduce(score, reduction)


def spectral_angle_mapper(
    preds: Tensor, target: Tensor, reduction: Literal["elementwise_mean", "sum", "none", None] = "elementwise_mean"
) -> Tensor:
    preds, target = _sam_update(preds, target)
    return _sam_compute(preds, target, reduction)
