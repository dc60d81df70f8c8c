"""Mean squared log error (API parity: reference ``functional/regression/log_mse.py:22-77``)."""
from typing import Tuple, Union

import torch
from torch import Tensor

from torchmetrics_forked_amd.functional.regression._common import _out_dtype, fused_sums
from torchmetrics_forked_amd.ops import regression as reg_ops
from torchmetrics_forked_amd.utilities.checks import _check_same_shape


def _mean_squared_log_error_update(preds: Tensor, target: Tensor) -> Tuple[Tensor, int]:
    _check_same_shape(preds, target)
    sums = fused_sums(preds, target, reg_ops.OP_SLE, flatten=True)
    if sums is not None:
        return sums[7, 0].to(_out_dtype(preds, target)), target.numel()
    return torch.sum(torch.pow(torch.log1p(preds) - torch.log1p(target), 2)), target.numel()


def _mean_squared_log_error_compute(sum_squared_log_error: Tensor, num_obs: Union[int, Tensor]) -> Tensor:
    return sum_squared_log_error / num_obs


def mean_squared_log_error(preds: Tensor, target: Tensor) -> Tensor:
    return _mean_squared_log_error_compute(*_mean_squared_log_error_update(preds, target))
