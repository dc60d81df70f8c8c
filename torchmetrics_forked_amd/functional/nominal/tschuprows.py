"""Tschuprow's T (API parity: reference ``functional/nominal/tschuprows.py:32-180``)."""
from typing import Optional

import torch
from torch import Tensor
from typing_extensions import Literal

from torchmetrics_forked_amd.functional.nominal.utils import (
    _compute_bias_corrected_values,
    _compute_chi_squared,
    _drop_empty_rows_and_cols,
    _nominal_input_validation,
    _nominal_update,
    _num_classes,
    _pairwise_matrix,
    _unable_to_use_bias_correction_warning,
)


def _tschuprows_t_update(preds: Tensor, target: Tensor, num_classes: int, nan_strategy: str = "replace",
                         nan_replace_value: Optional[float] = 0.0) -> Tensor:
    return _nominal_update(preds, target, num_classes, nan_strategy, nan_replace_value)


def _tschuprows_t_compute(confmat: Tensor, bias_correction: bool) -> Tensor:
    confmat = _drop_empty_rows_and_cols(confmat.float())
    cm_sum = confmat.sum()
    phi_squared = _compute_chi_squared(confmat, bias_correction) / cm_sum
    num_rows, num_cols = confmat.shape
    if bias_correction:
        phi_c, rows_c, cols_c = _compute_bias_corrected_values(phi_squared, num_rows, num_cols, cm_sum)
        if torch.min(rows_c, cols_c) == 1:
            _unable_to_use_bias_correction_warning(metric_name="Tschuprow's T")
            return torch.tensor(float("nan"), device=confmat.device)
        value = torch.sqrt(phi_c / torch.sqrt((rows_c - 1) * (cols_c - 1)))
    else:
        r = torch.tensor(num_rows, device=phi_squared.device)
        c = torch.tensor(num_cols, device=phi_squared.device)
        value = torch.sqrt(phi_squared / torch.sqrt((r - 1) * (c - 1)))
    return value.clamp(0.0, 1.0)


def tschuprows_t(
    preds: Tensor,
    target: Tensor,
    bias_correction: bool = True,
    nan_strategy: Literal["replace", "drop"] = "replace",
    nan_replace_value: Optional[float] = 0.0,
) -> Tensor:
    _nominal_input_validation(nan_strategy, nan_replace_value)
    confmat = _tschuprows_t_update(preds, target, _num_classes(preds, target), nan_strategy, nan_replace_value)
    return _tschuprows_t_compute(confmat, bias_correction)


def tschuprows_t_matrix(
    matrix: Tensor,
    bias_correction: bool = True,
    nan_strategy: Literal["replace", "drop"] = "replace",
    nan_replace_value: Optional[float] = 0.0,
) -> Tensor:
    _nominal_input_validation(nan_strategy, nan_replace_value)
    return _pairwise_matrix(matrix, lambda x, y: _tschuprows_t_compute(
        _tschuprows_t_update(x, y, _num_classes(x, y), nan_strategy, nan_replace_value), bias_correction))
