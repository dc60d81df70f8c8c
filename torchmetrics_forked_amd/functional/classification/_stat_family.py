"""Shared driver for every metric that is a reduction of (tp, fp, tn, fn).

Accuracy, precision, recall, F-beta, specificity and Hamming distance all run the same stat-scores engine and
differ only in the final reduction (reference ``accuracy.py:37-86``, ``precision_recall.py:37-57``,
``f_beta.py:37-57``, ``specificity.py``, ``hamming.py``).  One driver = one fused device pass per call.
"""
from typing import Callable, Optional

import torch
from torch import Tensor

from torchmetrics_forked_amd.functional.classification.stat_scores import (
    _binary_stat_scores_arg_validation,
    _binary_stat_scores_format,
    _binary_stat_scores_tensor_validation,
    _binary_stat_scores_update,
    _binary_stats_fused,
    _multiclass_stat_scores_arg_validation,
    _multiclass_stat_scores_tensor_validation,
    _multiclass_stat_scores_update,
    _multilabel_stat_scores_arg_validation,
    _multilabel_stat_scores_format,
    _multilabel_stat_scores_tensor_validation,
    _multilabel_stat_scores_update,
    _multilabel_stats_fused,
)
from torchmetrics_forked_amd.utilities.compute import _adjust_weights_safe_divide, _safe_divide
from torchmetrics_forked_amd.utilities.enums import ClassificationTask

Reducer = Callable[..., Tensor]


_AVG_CODE = {"binary": 0, "micro": 1, "macro": 2, "weighted": 3, "none": 4, None: 4}


def _host_reduce(kind: int, tp: Tensor, fp: Tensor, tn: Tensor, fn: Tensor, average: Optional[str], multidim_average: str,
                 multilabel: bool, beta: float = 1.0) -> Optional[Tensor]:
    """CPU int64 states: the whole reduction in one native call (csrc/host_classification.cpp ``stat_reduce_host``);
    ``None`` when it does not apply (device tensors, float states, autograd, no native library)."""
    if tp.is_cuda or tp.dtype != torch.long or average not in _AVG_CODE or tp.requires_grad:
        return None
    if average not in ("binary", "none", None):
        glob = multidim_average == "global"
        if not ((glob and tp.ndim == 1) or (not glob and tp.ndim == 2) or (glob and tp.ndim == 0 and average == "micro")):
            return None
    if not _native_loaded():
        return None
    if not (fp.dtype == tn.dtype == fn.dtype == torch.long and not (fp.is_cuda or tn.is_cuda or fn.is_cuda)):
        return None
    return torch.ops.tmx.stat_reduce_host(tp, fp, tn, fn, kind, _AVG_CODE[average], multilabel, float(beta))


_NATIVE = []


def _native_loaded() -> bool:
    if not _NATIVE:
        from torchmetrics_forked_amd import ops

        _NATIVE.append(bool(ops.load()))
    return _NATIVE[0]


def _sum_micro(x: Tensor, multidim_average: str) -> Tensor:
    return x.sum(dim=0 if multidim_average == "global" else 1)


def _accuracy_reduce(tp, fp, tn, fn, average, multidim_average="global", multilabel=False) -> Tensor:  # noqa: ANN001
    r = _host_reduce(0, tp, fp, tn, fn, average, multidim_average, multilabel)
    if r is not None:
        return r
    if average == "binary":
        return _safe_divide(tp + tn, tp + tn + fp + fn)
    if average == "micro":
        tp, fn = _sum_micro(tp, multidim_average), _sum_micro(fn, multidim_average)
        if multilabel:
            fp, tn = _sum_micro(fp, multidim_average), _sum_micro(tn, multidim_average)
            return _safe_divide(tp + tn, tp + tn + fp + fn)
        return _safe_divide(tp, tp + fn)
    score = _safe_divide(tp + tn, tp + tn + fp + fn) if multilabel else _safe_divide(tp, tp + fn)
    return _adjust_weights_safe_divide(score, average, multilabel, tp, fp, fn)


def _precision_recall_reduce(stat, tp, fp, tn, fn, average, multidim_average="global", multilabel=False) -> Tensor:  # noqa: ANN001
    r = _host_reduce(1 if stat == "precision" else 2, tp, fp, tn, fn, average, multidim_average, multilabel)
    if r is not None:
        return r
    other = fp if stat == "precision" else fn
    if average == "binary":
        return _safe_divide(tp, tp + other)
    if average == "micro":
        tp, other = _sum_micro(tp, multidim_average), _sum_micro(other, multidim_average)
        return _safe_divide(tp, tp + other)
    score = _safe_divide(tp, tp + other)
    return _adjust_weights_safe_divide(score, average, multilabel, tp, fp, fn)


def _fbeta_reduce(tp, fp, tn, fn, beta, average, multidim_average="global", multilabel=False) -> Tensor:  # noqa: ANN001
    r = _host_reduce(3, tp, fp, tn, fn, average, multidim_average, multilabel, beta)
    if r is not None:
        return r
    b2 = beta**2

    def f(tp_: Tensor, fp_: Tensor, fn_: Tensor) -> Tensor:
        return _safe_divide((1 + b2) * tp_, (1 + b2) * tp_ + b2 * fn_ + fp_)

    if average == "binary":
        return f(tp, fp, fn)
    if average == "micro":
        return f(_sum_micro(tp, multidim_average), _sum_micro(fp, multidim_average), _sum_micro(fn, multidim_average))
    return _adjust_weights_safe_divide(f(tp, fp, fn), average, multilabel, tp, fp, fn)


def _specificity_reduce(tp, fp, tn, fn, average, multidim_average="global", multilabel=False) -> Tensor:  # noqa: ANN001
    r = _host_reduce(4, tp, fp, tn, fn, average, multidim_average, multilabel)
    if r is not None:
        return r
    if average == "binary":
        return _safe_divide(tn, tn + fp)
    if average == "micro":
        tn, fp_ = _sum_micro(tn, multidim_average), _sum_micro(fp, multidim_average)
        return _safe_divide(tn, tn + fp_)
    return _adjust_weights_safe_divide(_safe_divide(tn, tn + fp), average, multilabel, tp, fp, fn)


def _hamming_distance_reduce(tp, fp, tn, fn, average, multidim_average="global", multilabel=False) -> Tensor:  # noqa: ANN001
    r = _host_reduce(5, tp, fp, tn, fn, average, multidim_average, multilabel)
    if r is not None:
        return r
    if average == "binary":
        return 1 - _safe_divide(tp + tn, tp + fp + tn + fn)
    if average == "micro":
        tp, fn = _sum_micro(tp, multidim_average), _sum_micro(fn, multidim_average)
        if multilabel:
            fp, tn = _sum_micro(fp, multidim_average), _sum_micro(tn, multidim_average)
            return 1 - _safe_divide(tp + tn, tp + tn + fp + fn)
        return 1 - _safe_divide(tp, tp + fn)
    score = 1 - _safe_divide(tp + tn, tp + tn + fp + fn) if multilabel else 1 - _safe_divide(tp, tp + fn)
    return _adjust_weights_safe_divide(score, average, multilabel, tp, fp, fn)


# ----------------------------------------------------------------------------------------------- drivers
def binary_family(
    reduce: Reducer,
    preds: Tensor,
    target: Tensor,
    threshold: float,
    multidim_average: str,
    ignore_index: Optional[int],
    validate_args: bool,
) -> Tensor:
    if validate_args:
        _binary_stat_scores_arg_validation(threshold, multidim_average, ignore_index)
        _binary_stat_scores_tensor_validation(preds, target, multidim_average, ignore_index)
    if multidim_average == "global":
        tp, fp, tn, fn = _binary_stats_fused(preds, target, threshold, ignore_index)
    else:
        p, t = _binary_stat_scores_format(preds, target, threshold, ignore_index)
        tp, fp, tn, fn = _binary_stat_scores_update(p, t, multidim_average)
    return reduce(tp, fp, tn, fn, average="binary", multidim_average=multidim_average)


def multiclass_family(
    reduce: Reducer,
    preds: Tensor,
    target: Tensor,
    num_classes: int,
    average: Optional[str],
    top_k: int,
    multidim_average: str,
    ignore_index: Optional[int],
    validate_args: bool,
) -> Tensor:
    if validate_args:
        _multiclass_stat_scores_arg_validation(num_classes, top_k, average, multidim_average, ignore_index)
        _multiclass_stat_scores_tensor_validation(preds, target, num_classes, multidim_average, ignore_index)
    tp, fp, tn, fn = _multiclass_stat_scores_update(preds, target, num_classes, top_k, average, multidim_average, ignore_index)
    return reduce(tp, fp, tn, fn, average=average, multidim_average=multidim_average)


def multilabel_family(
    reduce: Reducer,
    preds: Tensor,
    target: Tensor,
    num_labels: int,
    threshold: float,
    average: Optional[str],
    multidim_average: str,
    ignore_index: Optional[int],
    validate_args: bool,
) -> Tensor:
    if validate_args:
        _multilabel_stat_scores_arg_validation(num_labels, threshold, average, multidim_average, ignore_index)
        _multilabel_stat_scores_tensor_validation(preds, target, num_labels, multidim_average, ignore_index)
    if multidim_average == "global":
        tp, fp, tn, fn = _multilabel_stats_fused(preds, target, num_labels, threshold, ignore_index)
    else:
        p, t = _multilabel_stat_scores_format(preds, target, num_labels, threshold, ignore_index)
        tp, fp, tn, fn = _multilabel_stat_scores_update(p, t, multidim_average)
    return reduce(tp, fp, tn, fn, average=average, multidim_average=multidim_average, multilabel=True)


def task_dispatch(
    task: str,
    binary_fn: Callable[..., Tensor],
    multiclass_fn: Callable[..., Tensor],
    multilabel_fn: Callable[..., Tensor],
    num_classes: Optional[int],
    num_labels: Optional[int],
    top_k: Optional[int] = 1,
    check_top_k: bool = True,
) -> Callable[..., Tensor]:
    """Validate the task-specific integer arguments and return the concrete function."""
    t = ClassificationTask.from_str(task)
    if t == ClassificationTask.BINARY:
        return binary_fn
    if t == ClassificationTask.MULTICLASS:
        if not isinstance(num_classes, int):
            raise ValueError(f"`num_classes` is expected to be `int` but `{type(num_classes)} was passed.`")
        if check_top_k and not isinstance(top_k, int):
            raise ValueError(f"`top_k` is expected to be `int` but `{type(top_k)} was passed.`")
        return multiclass_fn
    if t == ClassificationTask.MULTILABEL:
        if not isinstance(num_labels, int):
            raise ValueError(f"`num_labels` is expected to be `int` but `{type(num_labels)} was passed.`")
        return multilabel_fn
    raise ValueError(f"Unsupported task `{task}`")
