"""Shared nominal-association helpers (behavioural parity: reference ``functional/nominal/utils.py:20-110``).

Contingency tables come from the framework's confusion-matrix kernel (LDS-privatised histogram on the GPU)."""
from typing import Optional, Tuple

import torch
from torch import Tensor
from typing_extensions import Literal

from torchmetrics_forked_amd.ops import classification as cls_ops
from torchmetrics_forked_amd.utilities.prints import rank_zero_warn


def _nominal_input_validation(nan_strategy: str, nan_replace_value: Optional[float]) -> None:
    if nan_strategy not in ("replace", "drop"):
        raise ValueError(
            f"Argument `nan_strategy` is expected to be one of `['replace', 'drop']`, but got {nan_strategy}"
        )
    if nan_strategy == "replace" and not isinstance(nan_replace_value, (float, int)):
        raise ValueError(
            "Argument `nan_replace` is expected to be of a type `int` or `float` when `nan_strategy = 'replace`, "
            f"but got {nan_replace_value}"
        )


def _contingency(preds: Tensor, target: Tensor, num_classes: int) -> Tensor:
    """``[num_classes, num_classes]`` int64 table, rows = target category, cols = preds category."""
    confmat = torch.zeros(num_classes, num_classes, dtype=torch.long, device=target.device)
    cls_ops.mc_confmat_update(preds.reshape(-1).long(), target.reshape(-1).long(), confmat, None)
    return confmat


def _nominal_update(
    preds: Tensor, target: Tensor, num_classes: int, nan_strategy: str = "replace", nan_replace_value: Optional[float] = 0.0
) -> Tensor:
    preds = preds.argmax(1) if preds.ndim == 2 else preds
    target = target.argmax(1) if target.ndim == 2 else target
    preds, target = _handle_nan_in_data(preds, target, nan_strategy, nan_replace_value)
    return _contingency(preds, target, num_classes)


def _compute_expected_freqs(confmat: Tensor) -> Tensor:
    return torch.outer(confmat.sum(1), confmat.sum(0)) / confmat.sum()


def _compute_chi_squared(confmat: Tensor, bias_correction: bool) -> Tensor:
    confmat = confmat.float() if not confmat.is_floating_point() else confmat.clone()
    expected = _compute_expected_freqs(confmat)
    df = expected.numel() - sum(expected.shape) + expected.ndim - 1
    if df == 0:
        return torch.tensor(0.0, device=confmat.device)
    if df == 1 and bias_correction:
        direction = (expected - confmat).sign()
        confmat = confmat + direction * torch.minimum(0.5 * torch.ones_like(direction), direction.abs())
    return torch.sum((confmat - expected) ** 2 / expected)


def _drop_empty_rows_and_cols(confmat: Tensor) -> Tensor:
    confmat = confmat[confmat.sum(1) != 0]
    return confmat[:, confmat.sum(0) != 0]


def _compute_phi_squared_corrected(phi_squared: Tensor, num_rows: int, num_cols: int, confmat_sum: Tensor) -> Tensor:
    return torch.clamp(phi_squared - (num_rows - 1) * (num_cols - 1) / (confmat_sum - 1), min=0.0)


def _compute_rows_and_cols_corrected(num_rows: int, num_cols: int, confmat_sum: Tensor) -> Tuple[Tensor, Tensor]:
    return num_rows - (num_rows - 1) ** 2 / (confmat_sum - 1), num_cols - (num_cols - 1) ** 2 / (confmat_sum - 1)


def _compute_bias_corrected_values(
    phi_squared: Tensor, num_rows: int, num_cols: int, confmat_sum: Tensor
) -> Tuple[Tensor, Tensor, Tensor]:
    phi = _compute_phi_squared_corrected(phi_squared, num_rows, num_cols, confmat_sum)
    rows, cols = _compute_rows_and_cols_corrected(num_rows, num_cols, confmat_sum)
    return phi, rows, cols


def _handle_nan_in_data(
    preds: Tensor, target: Tensor, nan_strategy: Literal["replace", "drop"] = "replace", nan_replace_value: Optional[float] = 0.0
) -> Tuple[Tensor, Tensor]:
    if nan_strategy == "replace":
        return preds.nan_to_num(nan_replace_value), target.nan_to_num(nan_replace_value)
    bad = preds.isnan() | target.isnan()
    return preds[~bad], target[~bad]


def _unable_to_use_bias_correction_warning(metric_name: str) -> None:
    rank_zero_warn(
        f"Unable to compute {metric_name} using bias correction. Please consider to set `bias_correction=False`."
    )


def _num_classes(x: Tensor, y: Tensor) -> int:
    return len(torch.cat([x, y]).unique())


def _pairwise_matrix(matrix: Tensor, fn) -> Tensor:  # noqa: ANN001
    """Symmetric ``[V, V]`` association matrix of all column pairs (diagonal 1)."""
    v = matrix.shape[1]
    out = torch.ones(v, v, device=matrix.device)
    for i in range(v):
        for j in range(i + 1, v):
            out[i, j] = out[j, i] = fn(matrix[:, i], matrix[:, j])
    return out
