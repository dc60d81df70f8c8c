"""Mean absolute error (API parity: reference ``functional/regression/mae.py:22-72``)."""
from typing import Tuple, Union

import torch
from torch import Tensor

from torchmetrics_forked_amd.functional.regression._common import _out_dtype, fused_sums
from torchmetrics_forked_amd.utilities.checks import _check_same_shape


def _mean_absolute_error_update(preds: Tensor, target: Tensor) -> Tuple[Tensor, int]:
    _check_same_shape(preds, target)
    sums = fused_sums(preds, target, flatten=True)
    if sums is not None:
        return sums[6, 0].to(_out_dtype(preds, target)), target.numel()
    return torch.sum(torch.abs(preds - target)), target.numel()


def _mean_absolute_error_compute(sum_abs_error: Tensor, num_obs: Union[int, Tensor]) -> Tensor:
    return sum_abs_error / num_obs


def mean_absolute_error(preds: Tensor, target: Tensor) -> Tensor:
    return _mean_absolute_error_compute(*_mean_absolute_error_update(preds, target))
