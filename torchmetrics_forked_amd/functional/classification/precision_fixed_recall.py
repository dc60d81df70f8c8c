"""Precision at fixed recall (API parity: reference ``functional/classification/precision_fixed_recall.py:47-390``)."""
from typing import List, Optional, Tuple, Union

import torch
from torch import Tensor
from typing_extensions import Literal

from torchmetrics_forked_amd.functional.classification.precision_recall_curve import (
    _adjust_threshold_arg,
    _binary_precision_recall_curve_tensor_validation,
    _multiclass_precision_recall_curve_tensor_validation,
    _multilabel_precision_recall_curve_tensor_validation,
    binary_curve_update,
    multiclass_curve_update,
    multilabel_curve_update,
)
from torchmetrics_forked_amd.functional.classification.recall_fixed_precision import (
    _binary_recall_at_fixed_precision_arg_validation,
    _fixed_compute,
    _lexargmax,
    _multiclass_recall_at_fixed_precision_arg_validation,
    _multilabel_recall_at_fixed_precision_arg_validation,
    _zip,
)
from torchmetrics_forked_amd.utilities.enums import ClassificationTask


def _precision_at_recall(precision: Tensor, recall: Tensor, thresholds: Tensor, min_recall: float) -> Tuple[Tensor, Tensor]:
    """Lexicographic max over (precision, recall, threshold) among points with ``recall >= min_recall``."""
    z = _zip(precision, recall, thresholds)
    z = z[z[:, 1] >= min_recall]
    if z.shape[0] > 0:
        max_precision, _, best_threshold = z[_lexargmax(z)[0]]
    else:
        max_precision = torch.tensor(0.0, device=precision.device, dtype=precision.dtype)
        best_threshold = torch.tensor(0)
    if max_precision == 0.0:
        best_threshold = torch.tensor(1e6, device=thresholds.device, dtype=thresholds.dtype)
    return max_precision, best_threshold


def binary_precision_at_fixed_recall(
    preds: Tensor,
    target: Tensor,
    min_recall: float,
    thresholds: Optional[Union[int, List[float], Tensor]] = None,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tuple[Tensor, Tensor]:
    if validate_args:
        _binary_recall_at_fixed_precision_arg_validation(min_recall, thresholds, ignore_index)
        _binary_precision_recall_curve_tensor_validation(preds, target, ignore_index)
    thr = _adjust_threshold_arg(thresholds, preds.device)
    state = binary_curve_update(preds, target, thr, ignore_index)
    return _fixed_compute(state, "binary", 1, thr, ignore_index, min_recall, _precision_at_recall)


def multiclass_precision_at_fixed_recall(
    preds: Tensor,
    target: Tensor,
    num_classes: int,
    min_recall: float,
    thresholds: Optional[Union[int, List[float], Tensor]] = None,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tuple[Tensor, Tensor]:
    if validate_args:
        _multiclass_recall_at_fixed_precision_arg_validation(num_classes, min_recall, thresholds, ignore_index)
        _multiclass_precision_recall_curve_tensor_validation(preds, target, num_classes, ignore_index)
    thr = _adjust_threshold_arg(thresholds, preds.device)
    state = multiclass_curve_update(preds, target, num_classes, thr, ignore_index)
    return _fixed_compute(state, "multiclass", num_classes, thr, ignore_index, min_recall, _precision_at_recall)


def multilabel_precision_at_fixed_recall(
    preds: Tensor,
    target: Tensor,
    num_labels: int,
    min_recall: float,
    thresholds: Optional[Union[int, List[float], Tensor]] = None,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tuple[Tensor, Tensor]:
    if validate_args:
        _multilabel_recall_at_fixed_precision_arg_validation(num_labels, min_recall, thresholds, ignore_index)
        _multilabel_precision_recall_curve_tensor_validation(preds, target, num_labels, ignore_index)
    thr = _adjust_threshold_arg(thresholds, preds.device)
    state = multilabel_curve_update(preds, target, num_labels, thr, ignore_index)
    return _fixed_compute(state, "multilabel", num_labels, thr, ignore_index, min_recall, _precision_at_recall)


def precision_at_fixed_recall(
    preds: Tensor,
    target: Tensor,
    task: Literal["binary", "multiclass", "multilabel"],
    min_recall: float,
    thresholds: Optional[Union[int, List[float], Tensor]] = None,
    num_classes: Optional[int] = None,
    num_labels: Optional[int] = None,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Optional[Tuple[Tensor, Tensor]]:
    task = ClassificationTask.from_str(task)
    if task == ClassificationTask.BINARY:
        return binary_precision_at_fixed_recall(preds, target, min_recall, thresholds, ignore_index, validate_args)
    if task == ClassificationTask.MULTICLASS:
        if not isinstance(num_classes, int):
            raise ValueError(f"`num_classes` is expected to be `int` but `{type(num_classes)} was passed.`")
        return multiclass_precision_at_fixed_recall(
            preds, target, num_classes, min_recall, thresholds, ignore_index, validate_args
        )
    if task == ClassificationTask.MULTILABEL:
        if not isinstance(num_labels, int):
            raise ValueError(f"`num_labels` is expected to be `int` but `{type(num_labels)} was passed.`")
        return multilabel_precision_at_fixed_recall(
            preds, target, num_labels, min_recall, thresholds, ignore_index, validate_args
        )
    return None
