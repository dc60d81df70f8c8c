"""Specificity (API parity: reference functional/classification/specificity.py:57-394).

Thin wrappers over the fused stat-scores engine in ``_stat_family``.
"""
from typing import Optional

from torch import Tensor
from typing_extensions import Literal

from torchmetrics_forked_amd.functional.classification._stat_family import (
    _specificity_reduce,
    binary_family,
    multiclass_family,
    multilabel_family,
    task_dispatch,
)


def binary_specificity(
    preds: Tensor,
    target: Tensor,
    threshold: float = 0.5,
    multidim_average: Literal["global", "samplewise"] = "global",
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """Binary specificity."""
    return binary_family(_specificity_reduce, preds, target, threshold, multidim_average, ignore_index, validate_args)


def multiclass_specificity(
    preds: Tensor,
    target: Tensor,
    num_classes: int,
    average: Optional[Literal["micro", "macro", "weighted", "none"]] = "macro",
    top_k: int = 1,
    multidim_average: Literal["global", "samplewise"] = "global",
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """Multiclass specificity."""
    return multiclass_family(
        _specificity_reduce, preds, target, num_classes, average, top_k, multidim_average, ignore_index, validate_args
    )


def multilabel_specificity(
    preds: Tensor,
    target: Tensor,
    num_labels: int,
    threshold: float = 0.5,
    average: Optional[Literal["micro", "macro", "weighted", "none"]] = "macro",
    multidim_average: Literal["global", "samplewise"] = "global",
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """Multilabel specificity."""
    return multilabel_family(
        _specificity_reduce, preds, target, num_labels, threshold, average, multidim_average, ignore_index, validate_args
    )


def specificity(
    preds: Tensor,
    target: Tensor,
    task: Literal["binary", "multiclass", "multilabel"],
    threshold: float = 0.5,
    num_classes: Optional[int] = None,
    num_labels: Optional[int] = None,
    average: Optional[Literal["micro", "macro", "weighted", "none"]] = "micro",
    multidim_average: Literal["global", "samplewise"] = "global",
    top_k: Optional[int] = 1,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """Task-dispatching specificity."""
    fn = task_dispatch(task, binary_specificity, multiclass_specificity, multilabel_specificity, num_classes, num_labels, top_k)
    if fn is binary_specificity:
        return fn(preds, target, threshold, multidim_average, ignore_index, validate_args)
    if fn is multiclass_specificity:
        return fn(preds, target, num_classes, average, top_k, multidim_average, ignore_index, validate_args)
    return fn(preds, target, num_labels, threshold, average, multidim_average, ignore_index, validate_args)
