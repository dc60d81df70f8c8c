"""Pearson's contingency coefficient (API parity: reference ``functional/nominal/pearson.py:29-150``)."""
from typing import Optional

import torch
from torch import Tensor
from typing_extensions import Literal

from torchmetrics_forked_amd.functional.nominal.utils import (
    _compute_chi_squared,
    _drop_empty_rows_and_cols,
    _nominal_input_validation,
    _nominal_update,
    _num_classes,
    _pairwise_matrix,
)


def _pearsons_contingency_coefficient_update(preds: Tensor, target: Tensor, num_classes: int, nan_strategy: str = "replace",
                                             nan_replace_value: Optional[float] = 0.0) -> Tensor:
    return _nominal_update(preds, target, num_classes, nan_strategy, nan_replace_value)


def _pearsons_contingency_coefficient_compute(confmat: Tensor) -> Tensor:
    confmat = _drop_empty_rows_and_cols(confmat.float())
    phi_squared = _compute_chi_squared(confmat, bias_correction=False) / confmat.sum()
    return torch.sqrt(phi_squared / (1 + phi_squared)).clamp(0.0, 1.0)


def pearsons_contingency_coefficient(
    preds: Tensor,
    target: Tensor,
    nan_strategy: Literal["replace", "drop"] = "replace",
    nan_replace_value: Optional[float] = 0.0,
) -> Tensor:
    _nominal_input_validation(nan_strategy, nan_replace_value)
    confmat = _pearsons_contingency_coefficient_update(preds, target, _num_classes(preds, target), nan_strategy, nan_replace_value)
    return _pearsons_contingency_coefficient_compute(confmat)


def pearsons_contingency_coefficient_matrix(
    matrix: Tensor,
    nan_strategy: Literal["replace", "drop"] = "replace",
    nan_replace_value: Optional[float] = 0.0,
) -> Tensor:
    _nominal_input_validation(nan_strategy, nan_replace_value)
    return _pairwise_matrix(matrix, lambda x, y: _pearsons_contingency_coefficient_compute(
        _pearsons_contingency_coefficient_update(x, y, _num_classes(x, y), nan_strategy, nan_replace_value)))
