"""Log-cosh error (API parity: reference ``functional/regression/log_cosh.py:22-93``)."""
from typing import Tuple

import torch
from torch import Tensor

from torchmetrics_forked_amd.functional.regression._common import _check_data_shape_to_num_outputs, _out_dtype, fused_sums
from torchmetrics_forked_amd.ops import regression as reg_ops
from torchmetrics_forked_amd.utilities.checks import _check_same_shape


def _unsqueeze_tensors(preds: Tensor, target: Tensor) -> Tuple[Tensor, Tensor]:
    if preds.ndim == 2:
        return preds, target
    return preds.unsqueeze(1), target.unsqueeze(1)


def _log_cosh_error_update(preds: Tensor, target: Tensor, num_outputs: int) -> Tuple[Tensor, Tensor]:
    _check_same_shape(preds, target)
    _check_data_shape_to_num_outputs(preds, target, num_outputs)
    preds, target = _unsqueeze_tensors(preds, target)
    num_obs = torch.tensor(target.shape[0], device=preds.device)
    sums = fused_sums(preds, target, reg_ops.OP_LOGCOSH)
    if sums is not None:
        return sums[7].to(_out_dtype(preds, target)).squeeze(), num_obs
    diff = preds - target
    return torch.log((torch.exp(diff) + torch.exp(-diff)) / 2).sum(0).squeeze(), num_obs


def _log_cosh_error_compute(sum_log_cosh_error: Tensor, num_obs: Tensor) -> Tensor:
    return (sum_log_cosh_error / num_obs).squeeze()


def log_cosh_error(preds: Tensor, target: Tensor) -> Tensor:
    s, n = _log_cosh_error_update(preds, target, num_outputs=1 if preds.ndim == 1 else preds.shape[-1])
    return _log_cosh_error_compute(s, n)
