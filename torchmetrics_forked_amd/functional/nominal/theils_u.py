"""Theil's U (uncertainty coefficient) (API parity: reference ``functional/nominal/theils_u.py:28-160``)."""
from typing import Optional

import torch
from torch import Tensor
from typing_extensions import Literal

from torchmetrics_forked_amd.functional.nominal.utils import (
    _drop_empty_rows_and_cols,
    _nominal_input_validation,
    _nominal_update,
    _num_classes,
    _pairwise_matrix,
)


def _conditional_entropy_compute(confmat: Tensor) -> Tensor:
    confmat = _drop_empty_rows_and_cols(confmat.float())
    total = confmat.sum()
    p_xy = confmat / total
    p_y = (confmat.sum(1) / total).unsqueeze(1).expand_as(p_xy)
    return torch.nansum(p_xy * torch.log(p_y / p_xy))


def _theils_u_update(preds: Tensor, target: Tensor, num_classes: int, nan_strategy: str = "replace",
                     nan_replace_value: Optional[float] = 0.0) -> Tensor:
    return _nominal_update(preds, target, num_classes, nan_strategy, nan_replace_value)


def _theils_u_compute(confmat: Tensor) -> Tensor:
    confmat = _drop_empty_rows_and_cols(confmat.float())
    s_xy = _conditional_entropy_compute(confmat)
    p_x = confmat.sum(0) / confmat.sum()
    s_x = -torch.sum(p_x * torch.log(p_x))
    if s_x == 0:
        return torch.tensor(0, device=confmat.device)
    return (s_x - s_xy) / s_x


def theils_u(
    preds: Tensor,
    target: Tensor,
    nan_strategy: Literal["replace", "drop"] = "replace",
    nan_replace_value: Optional[float] = 0.0,
) -> Tensor:
    confmat = _theils_u_update(preds, target, _num_classes(preds, target), nan_strategy, nan_replace_value)
    return _theils_u_compute(confmat)


def theils_u_matrix(
    matrix: Tensor,
    nan_strategy: Literal["replace", "drop"] = "replace",
    nan_replace_value: Optional[float] = 0.0,
) -> Tensor:
    _nominal_input_validation(nan_strategy, nan_replace_value)
    v = matrix.shape[1]
    out = torch.ones(v, v, device=matrix.device)
    for i in range(v):
        for j in range(v):
            if i != j:
                x, y = matrix[:, i], matrix[:, j]
                out[i, j] = _theils_u_compute(_theils_u_update(x, y, _num_classes(x, y), nan_strategy, nan_replace_value))
    return out
