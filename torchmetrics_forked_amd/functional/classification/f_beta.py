"""F-beta and F1 scores (API parity: reference functional/classification/f_beta.py:71-774)."""
from functools import partial
from typing import Optional

from torch import Tensor
from typing_extensions import Literal

from torchmetrics_forked_amd.functional.classification._stat_family import (
    _fbeta_reduce,
    binary_family,
    multiclass_family,
    multilabel_family,
    task_dispatch,
)


def _check_beta(beta: float) -> None:
    if not (isinstance(beta, float) and beta > 0):
        raise ValueError(f"Expected argument `beta` to be a float larger than 0, but got {beta}.")


def binary_fbeta_score(
    preds: Tensor,
    target: Tensor,
    beta: float,
    threshold: float = 0.5,
    multidim_average: Literal["global", "samplewise"] = "global",
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """Binary F-beta score."""
    if validate_args:
        _check_beta(beta)
    return binary_family(partial(_fbeta_reduce, beta=beta), preds, target, threshold, multidim_average, ignore_index, validate_args)


def multiclass_fbeta_score(
    preds: Tensor,
    target: Tensor,
    beta: float,
    num_classes: int,
    average: Optional[Literal["micro", "macro", "weighted", "none"]] = "macro",
    top_k: int = 1,
    multidim_average: Literal["global", "samplewise"] = "global",
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """Multiclass F-beta score."""
    if validate_args:
        _check_beta(beta)
    return multiclass_family(
        partial(_fbeta_reduce, beta=beta), preds, target, num_classes, average, top_k, multidim_average, ignore_index, validate_args
    )


def multilabel_fbeta_score(
    preds: Tensor,
    target: Tensor,
    beta: float,
    num_labels: int,
    threshold: float = 0.5,
    average: Optional[Literal["micro", "macro", "weighted", "none"]] = "macro",
    multidim_average: Literal["global", "samplewise"] = "global",
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """Multilabel F-beta score."""
    if validate_args:
        _check_beta(beta)
    return multilabel_family(
        partial(_fbeta_reduce, beta=beta), preds, target, num_labels, threshold, average, multidim_average, ignore_index, validate_args
    )


def binary_f1_score(
    preds: Tensor,
    target: Tensor,
    threshold: float = 0.5,
    multidim_average: Literal["global", "samplewise"] = "global",
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """Binary F1 score."""
    return binary_fbeta_score(preds, target, 1.0, threshold, multidim_average, ignore_index, validate_args)


def multiclass_f1_score(
    preds: Tensor,
    target: Tensor,
    num_classes: int,
    average: Optional[Literal["micro", "macro", "weighted", "none"]] = "macro",
    top_k: int = 1,
    multidim_average: Literal["global", "samplewise"] = "global",
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """Multiclass F1 score."""
    return multiclass_fbeta_score(preds, target, 1.0, num_classes, average, top_k, multidim_average, ignore_index, validate_args)


def multilabel_f1_score(
    preds: Tensor,
    target: Tensor,
    num_labels: int,
    threshold: float = 0.5,
    average: Optional[Literal["micro", "macro", "weighted", "none"]] = "macro",
    multidim_average: Literal["global", "samplewise"] = "global",
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """Multilabel F1 score."""
    return multilabel_fbeta_score(preds, target, 1.0, num_labels, threshold, average, multidim_average, ignore_index, validate_args)


def fbeta_score(
    preds: Tensor,
    target: Tensor,
    task: Literal["binary", "multiclass", "multilabel"],
    beta: float = 1.0,
    threshold: float = 0.5,
    num_classes: Optional[int] = None,
    num_labels: Optional[int] = None,
    average: Optional[Literal["micro", "macro", "weighted", "none"]] = "micro",
    multidim_average: Optional[Literal["global", "samplewise"]] = "global",
    top_k: Optional[int] = 1,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """Task-dispatching F-beta score."""
    fn = task_dispatch(task, binary_fbeta_score, multiclass_fbeta_score, multilabel_fbeta_score, num_classes, num_labels, top_k)
    if fn is binary_fbeta_score:
        return fn(preds, target, beta, threshold, multidim_average, ignore_index, validate_args)
    if fn is multiclass_fbeta_score:
        return fn(preds, target, beta, num_classes, average, top_k, multidim_average, ignore_index, validate_args)
    return fn(preds, target, beta, num_labels, threshold, average, multidim_average, ignore_index, validate_args)


def f1_score(
    preds: Tensor,
    target: Tensor,
    task: Literal["binary", "multiclass", "multilabel"],
    threshold: float = 0.5,
    num_classes: Optional[int] = None,
    num_labels: Optional[int] = None,
    average: Optional[Literal["micro", "macro", "weighted", "none"]] = "micro",
    multidim_average: Optional[Literal["global", "samplewise"]] = "global",
    top_k: Optional[int] = 1,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """Task-dispatching F1 score."""
    return fbeta_score(preds, target, task, 1.0, threshold, num_classes, num_labels, average, multidim_average, top_k, ignore_index, validate_args)
