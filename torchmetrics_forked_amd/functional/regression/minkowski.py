"""Minkowski distance (API parity: reference ``functional/regression/minkowski.py:22-80``)."""
import torch
from torch import Tensor

from torchmetrics_forked_amd.functional.regression._common import _out_dtype, fused_sums
from torchmetrics_forked_amd.ops import regression as reg_ops
from torchmetrics_forked_amd.utilities.checks import _check_same_shape
from torchmetrics_forked_amd.utilities.exceptions import TorchMetricsUserError


def _minkowski_distance_update(preds: Tensor, targets: Tensor, p: float) -> Tensor:
    _check_same_shape(preds, targets)
    if not (isinstance(p, (float, int)) and p >= 1):
        raise TorchMetricsUserError(f"Argument ``p`` must be a float or int greater than 1, but got {p}")
    sums = fused_sums(preds, targets, reg_ops.OP_MINKOWSKI, float(p), flatten=True)
    if sums is not None:
        return sums[7, 0].to(_out_dtype(preds, targets))
    return torch.sum(torch.pow(torch.abs(preds - targets), p))


def _minkowski_distance_compute(distance: Tensor, p: float) -> Tensor:
    return torch.pow(distance, 1.0 / p)


def minkowski_distance(preds: Tensor, targets: Tensor, p: float) -> Tensor:
    return _minkowski_distance_compute(_minkowski_distance_update(preds, targets, p), p)
