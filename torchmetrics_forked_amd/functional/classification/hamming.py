"""Hamming distance (API parity: reference functional/classification/hamming.py:86-429).

Thin wrappers over the fused stat-scores engine in ``_stat_family``.
"""
from typing import Optional

from torch import Tensor
from typing_extensions import Literal

from torchmetrics_forked_amd.functional.classification._stat_family import (
    _hamming_distance_reduce,
    binary_family,
    multiclass_family,
    multilabel_family,
    task_dispatch,
)


def binary_hamming_distance(
    preds: Tensor,
    target: Tensor,
    threshold: float = 0.5,
    multidim_average: Literal["global", "samplewise"] = "global",
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """Binary hamming distance."""
    return binary_family(_hamming_distance_reduce, preds, target, threshold, multidim_average, ignore_index, validate_args)


def multiclass_hamming_distance(
    preds: Tensor,
    target: Tensor,
    num_classes: int,
    average: Optional[Literal["micro", "macro", "weighted", "none"]] = "macro",
    top_k: int = 1,
    multidim_average: Literal["global", "samplewise"] = "global",
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """Multiclass hamming distance."""
    return multiclass_family(
        _hamming_distance_reduce, preds, target, num_classes, average, top_k, multidim_average, ignore_index, validate_args
    )


def multilabel_hamming_distance(
    preds: Tensor,
    target: Tensor,
    num_labels: int,
    threshold: float = 0.5,
    average: Optional[Literal["micro", "macro", "weighted", "none"]] = "macro",
    multidim_average: Literal["global", "samplewise"] = "global",
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """Multilabel hamming distance."""
    return multilabel_family(
        _hamming_distance_reduce, preds, target, num_labels, threshold, average, multidim_average, ignore_index, validate_args
    )


def hamming_distance(
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
    """Task-dispatching hamming distance."""
    fn = task_dispatch(task, binary_hamming_distance, multiclass_hamming_distance, multilabel_hamming_distance, num_classes, num_labels, top_k)
    if fn is binary_hamming_distance:
        return fn(preds, target, threshold, multidim_average, ignore_index, validate_args)
    if fn is multiclass_hamming_distance:
        return fn(preds, target, num_classes, average, top_k, multidim_average, ignore_index, validate_args)
    return fn(preds, target, num_labels, threshold, average, multidim_average, ignore_index, validate_args)
