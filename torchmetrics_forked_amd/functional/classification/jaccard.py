"""Jaccard index (API parity: reference ``functional/classification/jaccard.py``)."""
from typing import Optional

import torch
from torch import Tensor
from typing_extensions import Literal

from torchmetrics_forked_amd.functional.classification.confusion_matrix import (
    _binary_confusion_matrix_arg_validation,
    _binary_confusion_matrix_update,
    _multiclass_confusion_matrix_arg_validation,
    _multiclass_confusion_matrix_update,
    _multilabel_confusion_matrix_arg_validation,
    _multilabel_confusion_matrix_update,
)
from torchmetrics_forked_amd.functional.classification.stat_scores import (
    _binary_stat_scores_tensor_validation,
    _multiclass_stat_scores_tensor_validation,
    _multilabel_stat_scores_tensor_validation,
)
from torchmetrics_forked_amd.utilities.compute import _safe_divide
from torchmetrics_forked_amd.utilities.enums import ClassificationTask

_AVG = ["binary", "micro", "macro", "weighted", "none", None]


def _jaccard_index_reduce(confmat: Tensor, average: Optional[str], ignore_index: Optional[int] = None) -> Tensor:
    if average not in _AVG:
        raise ValueError(f"The `average` has to be one of {_AVG}, got {average}.")
    confmat = confmat.float()
    if average == "binary":
        return confmat[1, 1] / (confmat[0, 1] + confmat[1, 0] + confmat[1, 1])
    ignore_in = ignore_index is not None and 0 <= ignore_index < confmat.shape[0]
    multilabel = confmat.ndim == 3
    if multilabel:
        num = confmat[:, 1, 1]
        denom = confmat[:, 1, 1] + confmat[:, 0, 1] + confmat[:, 1, 0]
    else:
        num = torch.diag(confmat)
        denom = confmat.sum(0) + confmat.sum(1) - num
    if average == "micro":
        num = num.sum()
        denom = denom.sum() - (denom[ignore_index] if ignore_in else 0.0)
    jaccard = _safe_divide(num, denom)
    if average is None or average in ("none", "micro"):
        return jaccard
    if average == "weighted":
        weights = confmat[:, 1, 1] + confmat[:, 1, 0] if multilabel else confmat.sum(1)
    else:
        weights = torch.ones_like(jaccard)
        if ignore_in:
            weights[ignore_index] = 0.0
        if not multilabel:
            weights[confmat.sum(1) + confmat.sum(0) == 0] = 0.0
    return ((weights * jaccard) / weights.sum()).sum()


def _check_avg(average: Optional[str]) -> None:
    allowed = ("micro", "macro", "weighted", "none", None)
    if average not in allowed:
        raise ValueError(f"Expected argument `average` to be one of {allowed}, but got {average}.")


def binary_jaccard_index(
    preds: Tensor, target: Tensor, threshold: float = 0.5, ignore_index: Optional[int] = None, validate_args: bool = True
) -> Tensor:
    if validate_args:
        _binary_confusion_matrix_arg_validation(threshold, ignore_index)
        _binary_stat_scores_tensor_validation(preds, target, "global", ignore_index)
    return _jaccard_index_reduce(_binary_confusion_matrix_update(preds, target, threshold, ignore_index), average="binary")


def multiclass_jaccard_index(
    preds: Tensor,
    target: Tensor,
    num_classes: int,
    average: Optional[Literal["micro", "macro", "weighted", "none"]] = "macro",
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    if validate_args:
        _multiclass_confusion_matrix_arg_validation(num_classes, ignore_index)
        _check_avg(average)
        _multiclass_stat_scores_tensor_validation(preds, target, num_classes, "global", ignore_index)
    confmat = _multiclass_confusion_matrix_update(preds, target, num_classes, ignore_index)
    return _jaccard_index_reduce(confmat, average=average, ignore_index=ignore_index)


def multilabel_jaccard_index(
    preds: Tensor,
    target: Tensor,
    num_labels: int,
    threshold: float = 0.5,
    average: Optional[Literal["micro", "macro", "weighted", "none"]] = "macro",
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    if validate_args:
        _multilabel_confusion_matrix_arg_validation(num_labels, threshold, ignore_index)
        _check_avg(average)
        _multilabel_stat_scores_tensor_validation(preds, target, num_labels, "global", ignore_index)
    confmat = _multilabel_confusion_matrix_update(preds, target, num_labels, threshold, ignore_index)
    return _jaccard_index_reduce(confmat, average=average, ignore_index=ignore_index)


def jaccard_index(
    preds: Tensor,
    target: Tensor,
    task: Literal["binary", "multiclass", "multilabel"],
    threshold: float = 0.5,
    num_classes: Optional[int] = None,
    num_labels: Optional[int] = None,
    average: Optional[Literal["micro", "macro", "weighted", "none"]] = "macro",
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    task = ClassificationTask.from_str(task)
    if task == ClassificationTask.BINARY:
        return binary_jaccard_index(preds, target, threshold, ignore_index, validate_args)
    if task == ClassificationTask.MULTICLASS:
        if not isinstance(num_classes, int):
            raise ValueError(f"`num_classes` is expected to be `int` but `{type(num_classes)} was passed.`")
        return multiclass_jaccard_index(preds, target, num_classes, average, ignore_index, validate_args)
    if not isinstance(num_labels, int):
        raise ValueError(f"`num_labels` is expected to be `int` but `{type(num_labels)} was passed.`")
    return multilabel_jaccard_index(preds, target, num_labels, threshold, average, ignore_index, validate_args)
