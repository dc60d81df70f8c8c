"""Specificity at sensitivity (API parity: reference ``functional/classification/specificity_sensitivity.py:42-445``).

ROC from the curve engine, ``specificity = 1 - fpr``, then the best specificity among points whose sensitivity
(tpr) reaches ``min_sensitivity``.  ``specicity_at_sensitivity`` keeps the reference's misspelt public name.
"""
from typing import List, Optional, Tuple, Union

import torch
from torch import Tensor
from typing_extensions import Literal

from torchmetrics_forked_amd.functional.classification.precision_recall_curve import (
    _adjust_threshold_arg,
    _binary_precision_recall_curve_arg_validation,
    _binary_precision_recall_curve_tensor_validation,
    _multiclass_precision_recall_curve_arg_validation,
    _multiclass_precision_recall_curve_tensor_validation,
    _multilabel_precision_recall_curve_arg_validation,
    _multilabel_precision_recall_curve_tensor_validation,
    binary_curve_update,
    multiclass_curve_update,
    multilabel_curve_update,
)
from torchmetrics_forked_amd.functional.classification.recall_fixed_precision import _fixed_compute
from torchmetrics_forked_amd.functional.classification.roc import roc_compute
from torchmetrics_forked_amd.utilities.enums import ClassificationTask


def _convert_fpr_to_specificity(fpr: Tensor) -> Tensor:
    return 1 - fpr


def _specificity_at_sensitivity(
    specificity: Tensor, sensitivity: Tensor, thresholds: Tensor, min_sensitivity: float
) -> Tuple[Tensor, Tensor]:
    keep = sensitivity >= min_sensitivity
    if not keep.any():
        return (
            torch.tensor(0.0, device=specificity.device, dtype=specificity.dtype),
            torch.tensor(1e6, device=thresholds.device, dtype=thresholds.dtype),
        )
    specificity, thresholds = specificity[keep], thresholds[keep]
    idx = torch.argmax(specificity)
    return specificity[idx], thresholds[idx]


def _from_fpr(fpr: Tensor, tpr: Tensor, thr: Tensor, min_sensitivity: float) -> Tuple[Tensor, Tensor]:
    return _specificity_at_sensitivity(_convert_fpr_to_specificity(fpr), tpr, thr, min_sensitivity)


def _check_sensitivity(min_sensitivity: float) -> None:
    if not isinstance(min_sensitivity, float) and not (0 <= min_sensitivity <= 1):
        raise ValueError(
            f"Expected argument `min_sensitivity` to be an float in the [0,1] range, but got {min_sensitivity}"
        )


def _binary_specificity_at_sensitivity_arg_validation(
    min_sensitivity: float, thresholds: Optional[Union[int, List[float], Tensor]] = None, ignore_index: Optional[int] = None
) -> None:
    _binary_precision_recall_curve_arg_validation(thresholds, ignore_index)
    _check_sensitivity(min_sensitivity)


def _multiclass_specificity_at_sensitivity_arg_validation(
    num_classes: int, min_sensitivity: float, thresholds: Optional[Union[int, List[float], Tensor]] = None,
    ignore_index: Optional[int] = None,
) -> None:
    _multiclass_precision_recall_curve_arg_validation(num_classes, thresholds, ignore_index)
    _check_sensitivity(min_sensitivity)


def _multilabel_specificity_at_sensitivity_arg_validation(
    num_labels: int, min_sensitivity: float, thresholds: Optional[Union[int, List[float], Tensor]] = None,
    ignore_index: Optional[int] = None,
) -> None:
    _multilabel_precision_recall_curve_arg_validation(num_labels, thresholds, ignore_index)
    _check_sensitivity(min_sensitivity)


def _spec_compute(state, task, num, thr, ignore_index, min_sensitivity):  # noqa: ANN001, ANN202
    return _fixed_compute(state, task, num, thr, ignore_index, min_sensitivity, _from_fpr, curve_fn=roc_compute)


def binary_specificity_at_sensitivity(
    preds: Tensor,
    target: Tensor,
    min_sensitivity: float,
    thresholds: Optional[Union[int, List[float], Tensor]] = None,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tuple[Tensor, Tensor]:
    if validate_args:
        _binary_specificity_at_sensitivity_arg_validation(min_sensitivity, thresholds, ignore_index)
        _binary_precision_recall_curve_tensor_validation(preds, target, ignore_index)
    thr = _adjust_threshold_arg(thresholds, preds.device)
    state = binary_curve_update(preds, target, thr, ignore_index)
    return _spec_compute(state, "binary", 1, thr, ignore_index, min_sensitivity)


def multiclass_specificity_at_sensitivity(
    preds: Tensor,
    target: Tensor,
    num_classes: int,
    min_sensitivity: float,
    thresholds: Optional[Union[int, List[float], Tensor]] = None,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tuple[Tensor, Tensor]:
    if validate_args:
        _multiclass_specificity_at_sensitivity_arg_validation(num_classes, min_sensitivity, thresholds, ignore_index)
        _multiclass_precision_recall_curve_tensor_validation(preds, target, num_classes, ignore_index)
    thr = _adjust_threshold_arg(thresholds, preds.device)
    state = multiclass_curve_update(preds, target, num_classes, thr, ignore_index)
    return _spec_compute(state, "multiclass", num_classes, thr, ignore_index, min_sensitivity)


def multilabel_specificity_at_sensitivity(
    preds: Tensor,
    target: Tensor,
    num_labels: int,
    min_sensitivity: float,
    thresholds: Optional[Union[int, List[float], Tensor]] = None,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tuple[Tensor, Tensor]:
    if validate_args:
        _multilabel_specificity_at_sensitivity_arg_validation(num_labels, min_sensitivity, thresholds, ignore_index)
        _multilabel_precision_recall_curve_tensor_validation(preds, target, num_labels, ignore_index)
    thr = _adjust_threshold_arg(thresholds, preds.device)
    state = multilabel_curve_update(preds, target, num_labels, thr, ignore_index)
    return _spec_compute(state, "multilabel", num_labels, thr, ignore_index, min_sensitivity)


def specificity_at_sensitivity(
    preds: Tensor,
    target: Tensor,
    task: Literal["binary", "multiclass", "multilabel"],
    min_sensitivity: float,
    thresholds: Optional[Union[int, List[float], Tensor]] = None,
    num_classes: Optional[int] = None,
    num_labels: Optional[int] = None,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Union[Tensor, Tuple[Tensor, Tensor, Tensor]]:
    task = ClassificationTask.from_str(task)
    if task == ClassificationTask.BINARY:
        return binary_specificity_at_sensitivity(preds, target, min_sensitivity, thresholds, ignore_index, validate_args)
    if task == ClassificationTask.MULTICLASS:
        if not isinstance(num_classes, int):
            raise ValueError(f"`num_classes` is expected to be `int` but `{type(num_classes)} was passed.`")
        return multiclass_specificity_at_sensitivity(
            preds, target, num_classes, min_sensitivity, thresholds, ignore_index, validate_args
        )
    if task == ClassificationTask.MULTILABEL:
        if not isinstance(num_labels, int):
            raise ValueError(f"`num_labels` is expected to be `int` but `{type(num_labels)} was passed.`")
        return multilabel_specificity_at_sensitivity(
            preds, target, num_labels, min_sensitivity, thresholds, ignore_index, validate_args
        )
    raise ValueError(f"Not handled value: {task}")


specicity_at_sensitivity = specificity_at_sensitivity
