"""Precision and recall (API parity: reference functional/classification/precision_recall.py:60-742).

Thin wrappers over the fused stat-scores engine in ``_stat_family``.
"""
from typing import Optional

from torch import Tensor
from typing_extensions import Literal

from torchmetrics_forked_amd.functional.classification._stat_family import (
    _precision_recall_reduce,
    binary_family,
    multiclass_family,
    multilabel_family,
    task_dispatch,
)
from functools import partial


def binary_precision(
    preds: Tensor,
    target: Tensor,
    threshold: float = 0.5,
    multidim_average: Literal["global", "samplewise"] = "global",
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """Binary precision."""
    return binary_family(partial(_precision_recall_reduce, "precision"), preds, target, threshold, multidim_average, ignore_index, validate_args)


def multiclass_precision(
    preds: Tensor,
    target: Tensor,
    num_classes: int,
    average: Optional[Literal["micro", "macro", "weighted", "none"]] = "macro",
    top_k: int = 1,
    multidim_average: Literal["global", "samplewise"] = "global",
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """Multiclass precision."""
    return multiclass_family(
        partial(_precision_recall_reduce, "precision"), preds, target, num_classes, average, top_k, multidim_average, ignore_index, validate_args
    )


def multilabel_precision(
    preds: Tensor,
    target: Tensor,
    num_labels: int,
    threshold: float = 0.5,
    average: Optional[Literal["micro", "macro", "weighted", "none"]] = "macro",
    multidim_average: Literal["global", "samplewise"] = "global",
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """Multilabel precision."""
    return multilabel_family(
        partial(_precision_recall_reduce, "precision"), preds, target, num_labels, threshold, average, multidim_average, ignore_index, validate_args
    )


def precision(
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
    """Task-dispatching precision."""
    fn = task_dispatch(task, binary_precision, multiclass_precision, multilabel_precision, num_classes, num_labels, top_k)
    if fn is binary_precision:
        return fn(preds, target, threshold, multidim_average, ignore_index, validate_args)
    if fn is multiclass_precision:
        return fn(preds, target, num_classes, average, top_k, multidim_average, ignore_index, validate_args)
    return fn(preds, target, num_labels, threshold, average, multidim_average, ignore_index, validate_args)


def binary_recall(
    preds: Tensor,
    target: Tensor,
    threshold: float = 0.5,
    multidim_average: Literal["global", "samplewise"] = "global",
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """Binary recall."""
    return binary_family(partial(_precision_recall_reduce, "recall"), preds, target, threshold, multidim_average, ignore_index, validate_args)


def multiclass_recall(
    preds: Tensor,
    target: Tensor,
    num_classes: int,
    average: Optional[Literal["micro", "macro", "weighted", "none"]] = "macro",
    top_k: int = 1,
    multidim_average: Literal["global", "samplewise"] = "global",
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """Multiclass recall."""
    return multiclass_family(
        partial(_precision_recall_reduce, "recall"), preds, target, num_classes, average, top_k, multidim_average, ignore_index, validate_args
    )


def multilabel_recall(
    preds: Tensor,
    target: Tensor,
    num_labels: int,
    threshold: float = 0.5,
    average: Optional[Literal["micro", "macro", "weighted", "none"]] = "macro",
    multidim_average: Literal["global", "samplewise"] = "global",
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """Multilabel recall."""
    return multilabel_family(
        partial(_precision_recall_reduce, "recall"), preds, target, num_labels, threshold, average, multidim_average, ignore_index, validate_args
    )


def recall(
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
    """Task-dispatching recall."""
    fn = task_dispatch(task, binary_recall, multiclass_recall, multilabel_recall, num_classes, num_labels, top_k)
    if fn is binary_recall:
        return fn(preds, target, threshold, multidim_average, ignore_index, validate_args)
    if fn is multiclass_recall:
        return fn(preds, target, num_classes, average, top_k, multidim_average, ignore_index, validate_args)
    return fn(preds, target, num_labels, threshold, average, multidim_average, ignore_index, validate_args)
