"""Receiver operating characteristic (API parity: reference ``functional/classification/roc.py:40-550``)."""
from typing import List, Optional, Tuple, Union

import torch
from torch import Tensor
from typing_extensions import Literal

from torchmetrics_forked_amd.functional.classification.precision_recall_curve import (
    CurveState,
    _adjust_threshold_arg,
    _binary_precision_recall_curve_arg_validation,
    _binary_precision_recall_curve_tensor_validation,
    _micro_state,
    _multiclass_precision_recall_curve_arg_validation,
    _multiclass_precision_recall_curve_tensor_validation,
    _multilabel_precision_recall_curve_arg_validation,
    _multilabel_precision_recall_curve_tensor_validation,
    _points,
    binary_curve_update,
    multiclass_curve_update,
    multilabel_curve_update,
)
from torchmetrics_forked_amd.utilities.compute import _safe_divide, interp, macro_interp_sum
from torchmetrics_forked_amd.utilities.enums import ClassificationTask
from torchmetrics_forked_amd.utilities.prints import rank_zero_warn


def _roc_from_points(fps: Tensor, tps: Tensor, thres: Tensor) -> Tuple[Tensor, Tensor, Tensor]:
    """Reference ``_binary_roc_compute`` (roc.py:40-80) on one (fps, tps, thresholds) triple."""
    tps = torch.cat([torch.zeros(1, dtype=tps.dtype, device=tps.device), tps])
    fps = torch.cat([torch.zeros(1, dtype=fps.dtype, device=fps.device), fps])
    thres = torch.cat([torch.ones(1, dtype=thres.dtype, device=thres.device), thres])
    if fps[-1] <= 0:
        rank_zero_warn(
            "No negative samples in targets, false positive value should be meaningless."
            " Returning zero tensor in false positive score",
            UserWarning,
        )
        fpr = torch.zeros_like(thres)
    else:
        fpr = fps / fps[-1]
    if tps[-1] <= 0:
        rank_zero_warn(
            "No positive samples in targets, true positive value should be meaningless."
            " Returning zero tensor in true positive score",
            UserWarning,
        )
        tpr = torch.zeros_like(thres)
    else:
        tpr = tps / tps[-1]
    return fpr, tpr, thres


def _roc_from_binned(cm: Tensor, thresholds: Tensor) -> Tuple[Tensor, Tensor, Tensor]:
    """``cm [T, C, 2, 2]`` -> fpr, tpr ``[C, T]`` (thresholds flipped, reference roc.py:162-172)."""
    tps, fps, fns, tns = cm[:, :, 1, 1], cm[:, :, 0, 1], cm[:, :, 1, 0], cm[:, :, 0, 0]
    tpr = _safe_divide(tps, tps + fns).flip(0).T
    fpr = _safe_divide(fps, fps + tns).flip(0).T
    return fpr, tpr, thresholds.flip(0)


def roc_compute(
    state: CurveState,
    task: str,
    num: int,
    thresholds: Optional[Tensor],
    ignore_index: Optional[int] = None,
    average: Optional[str] = None,
) -> Union[Tuple[Tensor, Tensor, Tensor], Tuple[List[Tensor], List[Tensor], List[Tensor]]]:
    if average == "micro":
        return roc_compute(_micro_state(state, task, num, ignore_index), "binary", 1, thresholds)
    if state[0] == "binned":
        fpr, tpr, thr = _roc_from_binned(state[1], thresholds)
        if task == "binary":
            return fpr[0], tpr[0], thr
        if average == "macro":
            return _macro_roc(list(fpr), list(tpr), [thr] * num, num)
        return fpr, tpr, thr
    res = [_roc_from_points(*p) for p in _points(state, task, num, ignore_index)]
    if task == "binary":
        return res[0]
    fprs, tprs, thrs = [r[0] for r in res], [r[1] for r in res], [r[2] for r in res]
    if average == "macro":
        return _macro_roc(fprs, tprs, thrs, num)
    return fprs, tprs, thrs


def _macro_roc(fprs: List[Tensor], tprs: List[Tensor], thrs: List[Tensor], num: int) -> Tuple[Tensor, Tensor, Tensor]:
    thres = torch.cat(thrs, dim=0).sort(descending=True).values
    mean_fpr = torch.cat(fprs, dim=0).sort().values
    mean_tpr = macro_interp_sum(mean_fpr, fprs, tprs)  # one launch on the GPU (csrc/interp.hip)
    if mean_tpr is None:
        mean_tpr = torch.zeros_like(mean_fpr)
        for i in range(num):
            mean_tpr += interp(mean_fpr, fprs[i], tprs[i])
    mean_tpr /= num
    return mean_fpr, mean_tpr, thres


def binary_roc(
    preds: Tensor,
    target: Tensor,
    thresholds: Optional[Union[int, List[float], Tensor]] = None,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tuple[Tensor, Tensor, Tensor]:
    """(fpr, tpr, thresholds) for a binary task."""
    if validate_args:
        _binary_precision_recall_curve_arg_validation(thresholds, ignore_index)
        _binary_precision_recall_curve_tensor_validation(preds, target, ignore_index)
    thr = _adjust_threshold_arg(thresholds, preds.device)
    return roc_compute(binary_curve_update(preds, target, thr, ignore_index), "binary", 1, thr)


def multiclass_roc(
    preds: Tensor,
    target: Tensor,
    num_classes: int,
    thresholds: Optional[Union[int, List[float], Tensor]] = None,
    average: Optional[Literal["micro", "macro"]] = None,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Union[Tuple[Tensor, Tensor, Tensor], Tuple[List[Tensor], List[Tensor], List[Tensor]]]:
    """One-vs-rest ROC curves for every class (or micro / macro averaged)."""
    if validate_args:
        _multiclass_precision_recall_curve_arg_validation(num_classes, thresholds, ignore_index, average)
        _multiclass_precision_recall_curve_tensor_validation(preds, target, num_classes, ignore_index)
    thr = _adjust_threshold_arg(thresholds, preds.device)
    state = multiclass_curve_update(preds, target, num_classes, thr, ignore_index)
    return roc_compute(state, "multiclass", num_classes, thr, ignore_index, average)


def multilabel_roc(
    preds: Tensor,
    target: Tensor,
    num_labels: int,
    thresholds: Optional[Union[int, List[float], Tensor]] = None,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Union[Tuple[Tensor, Tensor, Tensor], Tuple[List[Tensor], List[Tensor], List[Tensor]]]:
    """Per-label ROC curves."""
    if validate_args:
        _multilabel_precision_recall_curve_arg_validation(num_labels, thresholds, ignore_index)
        _multilabel_precision_recall_curve_tensor_validation(preds, target, num_labels, ignore_index)
    thr = _adjust_threshold_arg(thresholds, preds.device)
    state = multilabel_curve_update(preds, target, num_labels, thr, ignore_index)
    return roc_compute(state, "multilabel", num_labels, thr, ignore_index)


def roc(
    preds: Tensor,
    target: Tensor,
    task: Literal["binary", "multiclass", "multilabel"],
    thresholds: Optional[Union[int, List[float], Tensor]] = None,
    num_classes: Optional[int] = None,
    num_labels: Optional[int] = None,
    average: Optional[Literal["micro", "macro"]] = None,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Union[Tuple[Tensor, Tensor, Tensor], Tuple[List[Tensor], List[Tensor], List[Tensor]]]:
    task = ClassificationTask.from_str(task)
    if task == ClassificationTask.BINARY:
        return binary_roc(preds, target, thresholds, ignore_index, validate_args)
    if task == ClassificationTask.MULTICLASS:
        if not isinstance(num_classes, int):
            raise ValueError(f"`num_classes` is expected to be `int` but `{type(num_classes)} was passed.`")
        return multiclass_roc(preds, target, num_classes, thresholds, average, ignore_index, validate_args)
    if task == ClassificationTask.MULTILABEL:
        if not isinstance(num_labels, int):
            raise ValueError(f"`num_labels` is expected to be `int` but `{type(num_labels)} was passed.`")
        return multilabel_roc(preds, target, num_labels, thresholds, ignore_index, validate_args)
    raise ValueError(f"Task {task} not supported.")
