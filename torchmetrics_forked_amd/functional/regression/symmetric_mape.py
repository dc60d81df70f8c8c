"""Symmetric MAPE (API parity: reference ``functional/regression/symmetric_mape.py:22-93``)."""
from typing import Tuple, Union

import torch
from torch import Tensor

from torchmetrics_forked_amd.functional.regression._common import _out_dtype, fused_sums
from torchmetrics_forked_amd.ops import regression as reg_ops
from torchmetrics_forked_amd.utilities.checks import _check_same_shape


def _symmetric_mean_absolute_percentage_error_update(
    preds: Tensor, target: Tensor, epsilon: float = 1.17e-06
) -> Tuple[Tensor, int]:
    _check_same_shape(preds, target)
    sums = fused_sums(preds, target, reg_ops.OP_SAPE, flatten=True) if epsilon == 1.17e-06 else None
    if sums is not None:
        return sums[7, 0].to(_out_dtype(preds, target)), target.numel()
    abs_per_error = torch.abs(preds - target) / torch.clamp(torch.abs(target) + torch.abs(preds), min=epsilon)
    return 2 * torch.sum(abs_per_error), target.numel()


def _symmetric_mean_absolute_percentage_error_compute(sum_abs_per_error: Tensor, num_obs: Union[int, Tensor]) -> Tensor:
    return sum_abs_per_error / num_obs


def symmetric_mean_absolute_percentage_error(preds: Tensor, target: Tensor) -> Tensor:
    return _symmetric_mean_absolute_percentage_error_compute(*_symmetric_mean_absolute_percentage_error_update(preds, target))
