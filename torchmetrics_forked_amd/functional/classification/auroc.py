"""Area under the ROC curve (API parity: reference ``functional/classification/auroc.py:45-479``).

For exact (``thresholds=None``) states all classes are scored at once (``_curve_engine.hist_scores`` /
``samples_scores``): no per-class Python loop and no per-class host syncs (reference SURVEY §3.5).
"""
from typing import List, Optional, Union

import torch
from torch import Tensor
from typing_extensions import Literal

from torchmetrics_forked_amd.functional.classification import _curve_engine as eng
from torchmetrics_forked_amd import ops
from torchmetrics_forked_amd.ops import classification as cls_ops
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
    binary_curve_update,
    multiclass_curve_update,
    multilabel_curve_update,
)
from torchmetrics_forked_amd.functional.classification.roc import _roc_from_binned, roc_compute
from torchmetrics_forked_amd.utilities.compute import _auc_compute_without_check, _safe_divide
from torchmetrics_forked_amd.utilities.enums import ClassificationTask
from torchmetrics_forked_amd.utilities.prints import rank_zero_warn
from torchmetrics_forked_amd.utilities.validation import defer_host_check


class ExactScores(tuple):
    """``(auroc, ap, n_pos, n_neg)`` per class; ``summary`` (float64[8] on the device, or None) carries the class
    averages and warning flags computed in one native pass (``ops.classification.curve_summary``)."""

    summary: Optional[Tensor] = None

    @classmethod
    def of(cls, auc: Tensor, ap: Tensor, pos: Tensor, neg: Tensor, summary: Optional[Tensor] = None) -> "ExactScores":
        out = cls((auc, ap, pos, neg))
        out.summary = summary
        return out


def _reduce_auroc(
    res: Tensor,
    average: Optional[str],
    weights: Optional[Tensor] = None,
    what: str = "Average precision",
    summary: Optional[Tensor] = None,
    col: int = 0,
) -> Tensor:
    """Class average ignoring NaN classes, without host syncs: the NaN warning is a deferred host check and the
    averages are masked reductions (``nanmean`` / NaN-zeroed weighted sum) instead of boolean indexing.  With a
    native ``summary`` (column ``col``: 0 = AUROC, 1 = AP) the averages and the flag come from it directly."""
    if average is None or average == "none":
        return res
    if average not in ("macro", "weighted") or (average == "weighted" and weights is None and summary is None):
        raise ValueError("Received an incompatible combinations of inputs to make reduction.")

    def _warn(v: List[int]) -> None:
        if v[0]:
            rank_zero_warn(
                f"{what} score for one or more classes was `nan`. Ignoring these classes in {average}-average", UserWarning
            )

    if summary is not None:
        defer_host_check(summary[2 + col], _warn)
        i = 4 + 2 * col + (average == "weighted")
        v32 = cls_ops.summary_f32(summary, i) if res.dtype == torch.float32 else None
        return v32 if v32 is not None else summary[i].to(res.dtype)
    nan = torch.isnan(res)
    defer_host_check(nan.any(), _warn)
    if average == "macro":
        return torch.nanmean(res)
    w = torch.where(nan, torch.zeros_like(weights), weights.to(res.dtype))  # type: ignore[union-attr]
    w = _safe_divide(w, w.sum())
    return torch.where(nan, torch.zeros_like(res), res * w).sum()


def _warn_degenerate(P: Tensor, N: Tensor, summary: Optional[Tensor] = None) -> None:
    """Same warnings the reference emits from ``_binary_roc_compute`` for classes without pos/neg samples
    (flags read with the compute's other host checks)."""

    def _warn(flags: List[int]) -> None:
        if flags[0]:
            rank_zero_warn(
                "No negative samples in targets, false positive value should be meaningless."
                " Returning zero tensor in false positive score",
                UserWarning,
            )
        if flags[1]:
            rank_zero_warn(
                "No positive samples in targets, true positive value should be meaningless."
                " Returning zero tensor in true positive score",
                UserWarning,
            )

    flags = summary[0:2] if summary is not None else torch.stack([(N <= 0).any(), (P <= 0).any()])
    defer_host_check(flags, _warn)


def _exact_scores(state: CurveState, task: str, num: int, ignore_index: Optional[int]) -> ExactScores:
    """(auroc, ap, P, N) per class for hist / samples states (``.summary`` set on the native histogram path)."""
    if state[0] == "hist":
        sc, summ = cls_ops.curve_hist_scores(state[1], state[3] if len(state) > 3 else None, state[4] if len(state) > 4 else None)
        return ExactScores.of(sc[:, 0], sc[:, 1], sc[:, 2], sc[:, 3], summ)
    preds, target = state[1], state[2]
    anchored = eng.anchored_scores(preds, target, task, num, ignore_index)
    if anchored is not None:
        return ExactScores.of(anchored[:, 0], anchored[:, 1], anchored[:, 2], anchored[:, 3], cls_ops.curve_summary(anchored))
    radix = eng.sorted_scores(preds, target, task, ignore_index)  # GPU fp32 / fp64: csrc/radix.hip, no ATen sort
    if radix is not None:
        return ExactScores.of(radix[:, 0], radix[:, 1], radix[:, 2], radix[:, 3], cls_ops.curve_summary(radix))
    if isinstance(preds, eng.ColumnChunks):
        preds = preds.materialize()
    if task == "binary":
        return ExactScores.of(*eng.samples_scores(preds, target == 1))
    if task == "multiclass":
        if preds.device.type == "cpu" and preds.is_floating_point() and preds.ndim == 2 and ops.load():
            # host op with the class ids themselves (label = target == c): no [N, C] one-hot matrix
            out = torch.ops.tmx.curve_scores_host(preds.detach(), target.long(), None)
            return ExactScores.of(out[:, 0], out[:, 1], out[:, 2], out[:, 3])
        labels = torch.nn.functional.one_hot(target.long(), num).bool()
        return ExactScores.of(*eng.samples_scores(preds, labels))
    valid = None if ignore_index is None else target != ignore_index
    return ExactScores.of(*eng.samples_scores(preds, target == 1, valid))


def auroc_compute(
    state: CurveState,
    task: str,
    num: int,
    thresholds: Optional[Tensor],
    average: Optional[str] = "macro",
    max_fpr: Optional[float] = None,
    ignore_index: Optional[int] = None,
) -> Tensor:
    if task != "binary" and average == "micro":
        return auroc_compute(_micro_state(state, task, num, ignore_index), "binary", 1, thresholds, None, None)
    if task == "binary" and max_fpr is not None and max_fpr != 1:
        return _binary_partial_auroc(state, thresholds, max_fpr)
    if state[0] == "binned":
        fpr, tpr, _ = _roc_from_binned(state[1], thresholds)
        res = _auc_compute_without_check(fpr, tpr, 1.0, axis=1)
        if task == "binary":
            return res[0]
        weights = state[1][0, :, 1, :].sum(-1)
        return _reduce_auroc(res, average, weights)
    sc = _exact_scores(state, task, num, ignore_index)
    auc, _, P, N = sc
    _warn_degenerate(P, N, sc.summary)
    if task != "binary" and average in ("macro", "weighted") and sc.summary is not None:
        # the class average comes from the native summary: no per-class conversions
        return _reduce_auroc(auc[:0].to(torch.float32), average, None, summary=sc.summary, col=0)
    res = auc.to(torch.float32)
    if task == "binary":
        return res[0]
    return _reduce_auroc(res, average, P.to(torch.float32), summary=sc.summary, col=0)


def _binary_partial_auroc(state: CurveState, thresholds: Optional[Tensor], max_fpr: float) -> Tensor:
    fpr, tpr, _ = roc_compute(state, "binary", 1, thresholds)
    if fpr.sum() == 0 or tpr.sum() == 0:
        return _auc_compute_without_check(fpr, tpr, 1.0)
    max_area = torch.tensor(max_fpr, device=fpr.device)
    stop = torch.bucketize(max_area, fpr, out_int32=True, right=True)
    weight = (max_area - fpr[stop - 1]) / (fpr[stop] - fpr[stop - 1])
    interp_tpr = torch.lerp(tpr[stop - 1], tpr[stop], weight)
    tpr = torch.cat([tpr[:stop], interp_tpr.view(1)])
    fpr = torch.cat([fpr[:stop], max_area.view(1)])
    partial = _auc_compute_without_check(fpr, tpr, 1.0)
    min_area = 0.5 * max_area**2
    return 0.5 * (1 + (partial - min_area) / (max_area - min_area))


def _binary_auroc_arg_validation(
    max_fpr: Optional[float] = None,
    thresholds: Optional[Union[int, List[float], Tensor]] = None,
    ignore_index: Optional[int] = None,
) -> None:
    _binary_precision_recall_curve_arg_validation(thresholds, ignore_index)
    if max_fpr is not None and not isinstance(max_fpr, float) and 0 < max_fpr <= 1:
        raise ValueError(f"Arguments `max_fpr` should be a float in range (0, 1], but got: {max_fpr}")


def _multiclass_auroc_arg_validation(
    num_classes: int,
    average: Optional[str] = "macro",
    thresholds: Optional[Union[int, List[float], Tensor]] = None,
    ignore_index: Optional[int] = None,
) -> None:
    _multiclass_precision_recall_curve_arg_validation(num_classes, thresholds, ignore_index)
    allowed = ("macro", "weighted", "none", None)
    if average not in allowed:
        raise ValueError(f"Expected argument `average` to be one of {allowed} but got {average}")


def _multilabel_auroc_arg_validation(
    num_labels: int,
    average: Optional[str],
    thresholds: Optional[Union[int, List[float], Tensor]] = None,
    ignore_index: Optional[int] = None,
) -> None:
    _multilabel_precision_recall_curve_arg_validation(num_labels, thresholds, ignore_index)
    allowed = ("micro", "macro", "weighted", "none", None)
    if average not in allowed:
        raise ValueError(f"Expected argument `average` to be one of {allowed} but got {average}")


def binary_auroc(
    preds: Tensor,
    target: Tensor,
    max_fpr: Optional[float] = None,
    thresholds: Optional[Union[int, List[float], Tensor]] = None,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """Binary AUROC (optionally standardised partial AUC up to ``max_fpr``, McClish correction)."""
    if validate_args:
        _binary_auroc_arg_validation(max_fpr, thresholds, ignore_index)
        _binary_precision_recall_curve_tensor_validation(preds, target, ignore_index)
    thr = _adjust_threshold_arg(thresholds, preds.device)
    state = binary_curve_update(preds, target, thr, ignore_index)
    return auroc_compute(state, "binary", 1, thr, max_fpr=max_fpr)


def multiclass_auroc(
    preds: Tensor,
    target: Tensor,
    num_classes: int,
    average: Optional[Literal["macro", "weighted", "none"]] = "macro",
    thresholds: Optional[Union[int, List[float], Tensor]] = None,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """One-vs-rest multiclass AUROC."""
    if validate_args:
        _multiclass_auroc_arg_validation(num_classes, average, thresholds, ignore_index)
        _multiclass_precision_recall_curve_tensor_validation(preds, target, num_classes, ignore_index)
    thr = _adjust_threshold_arg(thresholds, preds.device)
    state = multiclass_curve_update(preds, target, num_classes, thr, ignore_index)
    return auroc_compute(state, "multiclass", num_classes, thr, average)


def multilabel_auroc(
    preds: Tensor,
    target: Tensor,
    num_labels: int,
    average: Optional[Literal["micro", "macro", "weighted", "none"]] = "macro",
    thresholds: Optional[Union[int, List[float], Tensor]] = None,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """Per-label AUROC, optionally averaged."""
    if validate_args:
        _multilabel_auroc_arg_validation(num_labels, average, thresholds, ignore_index)
        _multilabel_precision_recall_curve_tensor_validation(preds, target, num_labels, ignore_index)
    thr = _adjust_threshold_arg(thresholds, preds.device)
    state = multilabel_curve_update(preds, target, num_labels, thr, ignore_index)
    return auroc_compute(state, "multilabel", num_labels, thr, average, ignore_index=ignore_index)


def auroc(
    preds: Tensor,
    target: Tensor,
    task: Literal["binary", "multiclass", "multilabel"],
    thresholds: Optional[Union[int, List[float], Tensor]] = None,
    num_classes: Optional[int] = None,
    num_labels: Optional[int] = None,
    average: Optional[Literal["macro", "weighted", "none"]] = "macro",
    max_fpr: Optional[float] = None,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Optional[Tensor]:
    task = ClassificationTask.from_str(task)
    if task == ClassificationTask.BINARY:
        return binary_auroc(preds, target, max_fpr, thresholds, ignore_index, validate_args)
    if task == ClassificationTask.MULTICLASS:
        if not isinstance(num_classes, int):
            raise ValueError(f"`num_classes` is expected to be `int` but `{type(num_classes)} was passed.`")
        return multiclass_auroc(preds, target, num_classes, average, thresholds, ignore_index, validate_args)
    if task == ClassificationTask.MULTILABEL:
        if not isinstance(num_labels, int):
            raise ValueError(f"`num_labels` is expected to be `int` but `{type(num_labels)} was passed.`")
        return multilabel_auroc(preds, target, num_labels, average, thresholds, ignore_index, validate_args)
    return None
