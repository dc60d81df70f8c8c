"""Weighted MAPE (API parity: reference ``functional/regression/wmape.py:22-86``)."""
from typing import Tuple

import torch
from torch import Tensor

from torchmetrics_forked_amd.functional.regression._common import _out_dtype, fused_sums
from torchmetrics_forked_amd.ops import regression as reg_ops
from torchmetrics_forked_amd.utilities.checks import _check_same_shape


def _weighted_mean_absolute_percentage_error_update(preds: Tensor, target: Tensor) -> Tuple[Tensor, Tensor]:
    _check_same_shape(preds, target)
    sums = fused_sums(preds, target, reg_ops.OP_ABS_T, flatten=True)
    if sums is not None:
        dt = _out_dtype(preds, target)
        return sums[6, 0].to(dt), sums[7, 0].to(dt)
    return (preds - target).abs().sum(), target.abs().sum()


def _weighted_mean_absolute_percentage_error_compute(sum_abs_error: Tensor, sum_scale: Tensor, epsilon: float = 1.17e-06) -> Tensor:
    return sum_abs_error / torch.clamp(sum_scale, min=epsilon)


def weighted_mean_absolute_percentage_error(preds: Tensor, target: Tensor) -> Tensor:
    return _weighted_mean_absolute_percentage_error_compute(*_weighted_mean_absolute_percentage_error_update(preds, target))
