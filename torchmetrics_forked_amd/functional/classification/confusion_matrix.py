"""Confusion matrices (API parity: reference ``functional/classification/confusion_matrix.py:26-665``).

Engine B.  Binary ``[2, 2]`` and multilabel ``[L, 2, 2]`` matrices come from the fused tp/fp/tn/fn kernel
(one pass, LDS counters); multiclass ``[C, C]`` from the fused argmax + LDS-privatised histogram kernel.
"""
from typing import Optional

import torch
from torch import Tensor
from typing_extensions import Literal

from torchmetrics_forked_amd.functional.classification.stat_scores import (
    _binary_stat_scores_arg_validation,
    _binary_stat_scores_tensor_validation,
    _multiclass_stat_scores_tensor_validation,
    _multilabel_stat_scores_tensor_validation,
)
from torchmetrics_forked_amd.ops import classification as cls_ops
from torchmetrics_forked_amd.utilities.enums import ClassificationTask
from torchmetrics_forked_amd.utilities.prints import rank_zero_warn

_NORMALIZE = ("true", "pred", "all", "none", None)


def _confusion_matrix_reduce(confmat: Tensor, normalize: Optional[str] = None) -> Tensor:
    if normalize not in _NORMALIZE:
        raise ValueError(f"Argument `normalize` needs to one of the following: {_NORMALIZE}")
    if normalize is not None and normalize != "none":
        confmat = confmat if confmat.is_floating_point() else confmat.float()
        if normalize == "true":
            confmat = confmat / confmat.sum(dim=-1, keepdim=True)
        elif normalize == "pred":
            confmat = confmat / confmat.sum(dim=-2, keepdim=True)
        elif normalize == "all":
            confmat = confmat / confmat.sum(dim=[-2, -1], keepdim=True)
        nans = torch.isnan(confmat)
        n_nan = int(nans.sum())
        if n_nan:
            confmat[nans] = 0
            rank_zero_warn(f"{n_nan} NaN values found in confusion matrix have been replaced with zeros.")
    return confmat


def _check_normalize(normalize: Optional[str]) -> None:
    if normalize not in _NORMALIZE:
        raise ValueError(f"Expected argument `normalize` to be one of {_NORMALIZE}, but got {normalize}.")


def _binary_confusion_matrix_arg_validation(
    threshold: float = 0.5, ignore_index: Optional[int] = None, normalize: Optional[str] = None
) -> None:
    _binary_stat_scores_arg_validation(threshold, "global", ignore_index)
    _check_normalize(normalize)


def _multiclass_confusion_matrix_arg_validation(
    num_classes: int, ignore_index: Optional[int] = None, normalize: Optional[str] = None
) -> None:
    if not isinstance(num_classes, int) or num_classes < 2:
        raise ValueError(f"Expected argument `num_classes` to be an integer larger than 1, but got {num_classes}")
    if ignore_index is not None and not isinstance(ignore_index, int):
        raise ValueError(f"Expected argument `ignore_index` to either be `None` or an integer, but got {ignore_index}")
    _check_normalize(normalize)


def _multilabel_confusion_matrix_arg_validation(
    num_labels: int, threshold: float = 0.5, ignore_index: Optional[int] = None, normalize: Optional[str] = None
) -> None:
    if not isinstance(num_labels, int) or num_labels < 2:
        raise ValueError(f"Expected argument `num_labels` to be an integer larger than 1, but got {num_labels}")
    if not (isinstance(threshold, float) and (0 <= threshold <= 1)):
        raise ValueError(f"Expected argument `threshold` to be a float, but got {threshold}.")
    if ignore_index is not None and not isinstance(ignore_index, int):
        raise ValueError(f"Expected argument `ignore_index` to either be `None` or an integer, but got {ignore_index}")
    _check_normalize(normalize)


def _counts_to_confmat(counts: Tensor) -> Tensor:
    """``[L, 4]`` (tp, fp, tn, fn) -> ``[L, 2, 2]`` indexed [target][pred]."""
    tp, fp, tn, fn = counts.unbind(-1)
    return torch.stack([torch.stack([tn, fp], -1), torch.stack([fn, tp], -1)], -2)


def _binary_confusion_matrix_update(
    preds: Tensor, target: Tensor, threshold: float = 0.5, ignore_index: Optional[int] = None
) -> Tensor:
    counts = torch.zeros(1, 4, dtype=torch.long, device=target.device)
    cls_ops.binary_stats_update(preds, target, counts, 1, threshold, ignore_index)
    return _counts_to_confmat(counts)[0]


def _multiclass_confusion_matrix_update(
    preds: Tensor, target: Tensor, num_classes: int, ignore_index: Optional[int] = None
) -> Tensor:
    confmat = torch.zeros(num_classes, num_classes, dtype=torch.long, device=target.device)
    if preds.ndim == target.ndim + 1:
        preds = torch.movedim(preds, 1, -1).reshape(-1, num_classes)
    cls_ops.mc_confmat_update(preds, target.reshape(-1), confmat, ignore_index)
    return confmat


def _multilabel_confusion_matrix_update(
    preds: Tensor, target: Tensor, num_labels: int, threshold: float = 0.5, ignore_index: Optional[int] = None
) -> Tensor:
    counts = torch.zeros(num_labels, 4, dtype=torch.long, device=target.device)
    cls_ops.binary_stats_update(preds, target, counts, num_labels, threshold, ignore_index)
    return _counts_to_confmat(counts)


def binary_confusion_matrix(
    preds: Tensor,
    target: Tensor,
    threshold: float = 0.5,
    normalize: Optional[Literal["true", "pred", "all", "none"]] = None,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """``[2, 2]`` confusion matrix (rows = target, cols = prediction)."""
    if validate_args:
        _binary_confusion_matrix_arg_validation(threshold, ignore_index, normalize)
        _binary_stat_scores_tensor_validation(preds, target, "global", ignore_index)
    return _confusion_matrix_reduce(_binary_confusion_matrix_update(preds, target, threshold, ignore_index), normalize)


def multiclass_confusion_matrix(
    preds: Tensor,
    target: Tensor,
    num_classes: int,
    normalize: Optional[Literal["true", "pred", "all", "none"]] = None,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """``[C, C]`` confusion matrix; float ``[N, C, ...]`` preds are arg-maxed on device (fused)."""
    if validate_args:
        _multiclass_confusion_matrix_arg_validation(num_classes, ignore_index, normalize)
        _multiclass_stat_scores_tensor_validation(preds, target, num_classes, "global", ignore_index)
    return _confusion_matrix_reduce(_multiclass_confusion_matrix_update(preds, target, num_classes, ignore_index), normalize)


def multilabel_confusion_matrix(
    preds: Tensor,
    target: Tensor,
    num_labels: int,
    threshold: float = 0.5,
    normalize: Optional[Literal["true", "pred", "all", "none"]] = None,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """``[L, 2, 2]`` per-label confusion matrices."""
    if validate_args:
        _multilabel_confusion_matrix_arg_validation(num_labels, threshold, ignore_index, normalize)
        _multilabel_stat_scores_tensor_validation(preds, target, num_labels, "global", ignore_index)
    return _confusion_matrix_reduce(
        _multilabel_confusion_matrix_update(preds, target, num_labels, threshold, ignore_index), normalize
    )


def confusion_matrix(
    preds: Tensor,
    target: Tensor,
    task: Literal["binary", "multiclass", "multilabel"],
    threshold: float = 0.5,
    num_classes: Optional[int] = None,
    num_labels: Optional[int] = None,
    normalize: Optional[Literal["true", "pred", "all", "none"]] = None,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    task = ClassificationTask.from_str(task)
    if task == ClassificationTask.BINARY:
        return binary_confusion_matrix(preds, target, threshold, normalize, ignore_index, validate_args)
    if task == ClassificationTask.MULTICLASS:
        if not isinstance(num_classes, int):
            raise ValueError(f"`num_classes` is expected to be `int` but `{type(num_classes)} was passed.`")
        return multiclass_confusion_matrix(preds, target, num_classes, normalize, ignore_index, validate_args)
    if task == ClassificationTask.MULTILABEL:
        if not isinstance(num_labels, int):
            raise ValueError(f"`num_labels` is expected to be `int` but `{type(num_labels)} was passed.`")
        return multilabel_confusion_matrix(preds, target, num_labels, threshold, normalize, ignore_index, validate_args)
    raise ValueError(f"Task {task} not supported.")
