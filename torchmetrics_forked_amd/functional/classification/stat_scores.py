"""Stat-scores engine (tp / fp / tn / fn) for binary, multiclass and multilabel tasks.

Semantics follow reference ``functional/classification/stat_scores.py`` (binary :25-214, multiclass :217-562,
multilabel :565-817).  Execution differs:

* global statistics are accumulated by one fused HIP pass (``ops.classification.binary_stats_update`` for
  binary/multilabel, ``mc_confmat_update`` = fused argmax + LDS histogram for multiclass macro/weighted/none),
  instead of four compare-and-sum passes / an argmax + ``bincount`` pair;
* the sigmoid-if-out-of-[0,1] decision is a device-side flag (no host sync);
* tensor validation can be deferred to ``compute`` (``utilities.validation``).
"""
from typing import Optional, Tuple

import torch
from torch import Tensor
from typing_extensions import Literal

from torchmetrics_forked_amd import ops
from torchmetrics_forked_amd.ops import classification as cls_ops
from torchmetrics_forked_amd.utilities.checks import _check_same_shape
from torchmetrics_forked_amd.utilities.data import select_topk
from torchmetrics_forked_amd.utilities.enums import ClassificationTask
from torchmetrics_forked_amd.utilities.validation import DeferredChecks, fail_if

_AVERAGES = ("micro", "macro", "weighted", "none", None)
_MDMC = ("global", "samplewise")


# ---------------------------------------------------------------------------------------------------------
# shared argument checks
# ---------------------------------------------------------------------------------------------------------
def _check_threshold(threshold: float) -> None:
    if not (isinstance(threshold, float) and (0 <= threshold <= 1)):
        raise ValueError(f"Expected argument `threshold` to be a float in the [0,1] range, but got {threshold}.")


def _check_mdmc(multidim_average: str) -> None:
    if multidim_average not in _MDMC:
        raise ValueError(f"Expected argument `multidim_average` to be one of {_MDMC}, but got {multidim_average}")


def _check_ignore(ignore_index: Optional[int]) -> None:
    if ignore_index is not None and not isinstance(ignore_index, int):
        raise ValueError(f"Expected argument `ignore_index` to either be `None` or an integer, but got {ignore_index}")


def _check_average(average: Optional[str], allowed: tuple = _AVERAGES) -> None:
    if average not in allowed:
        raise ValueError(f"Expected argument `average` to be one of {allowed}, but got {average}")


def _check_binary_values(x: Tensor, name: str, ignore_index: Optional[int], sink: Optional[DeferredChecks], label: bool) -> None:
    bad = (x != 0) & (x != 1)
    if ignore_index is not None and not label:
        bad &= x != ignore_index
    if label:
        msg = lambda: (  # noqa: E731
            f"Detected the following values in `{name}`: {torch.unique(x)} but expected only"
            " the following values [0,1] since `preds` is a label tensor."
        )
    else:
        msg = lambda: (  # noqa: E731
            f"Detected the following values in `{name}`: {torch.unique(x)} but expected only"
            f" the following values {[0, 1] if ignore_index is None else [ignore_index]}."
        )
    fail_if(bad, RuntimeError, msg, sink, f"Detected values in `{name}` outside the allowed set.")


# ---------------------------------------------------------------------------------------------------------
# binary
# ---------------------------------------------------------------------------------------------------------
def _binary_stat_scores_arg_validation(
    threshold: float = 0.5, multidim_average: str = "global", ignore_index: Optional[int] = None
) -> None:
    _check_threshold(threshold)
    _check_mdmc(multidim_average)
    _check_ignore(ignore_index)


def _binary_stat_scores_tensor_validation(
    preds: Tensor,
    target: Tensor,
    multidim_average: str = "global",
    ignore_index: Optional[int] = None,
    sink: Optional[DeferredChecks] = None,
    check_values: bool = True,
) -> None:
    _check_same_shape(preds, target)
    if check_values:
        _check_binary_values(target, "target", ignore_index, sink, label=False)
        if not preds.is_floating_point():
            _check_binary_values(preds, "preds", None, sink, label=True)
    if multidim_average != "global" and preds.ndim < 2:
        raise ValueError("Expected input to be at least 2D when multidim_average is set to `samplewise`")


def _binary_stat_scores_format(
    preds: Tensor, target: Tensor, threshold: float = 0.5, ignore_index: Optional[int] = None
) -> Tuple[Tensor, Tensor]:
    """Labels ``[N, X]``; ignored targets become -1 (reference semantics)."""
    if preds.is_floating_point():
        flag = cls_ops.range_flag(preds).bool()
        preds = torch.where(flag, preds.sigmoid(), preds) > threshold
    preds = preds.reshape(preds.shape[0], -1)
    target = target.reshape(target.shape[0], -1)
    if ignore_index is not None:
        target = torch.where(target == ignore_index, torch.full_like(target, -1), target)
    return preds, target


def _samplewise_counts(preds: Tensor, target: Tensor, sum_dim) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    eq = target == preds
    pos = target == 1
    neg = target == 0
    tp = (eq & pos).sum(sum_dim).squeeze()
    fn = ((~eq) & pos).sum(sum_dim).squeeze()
    fp = ((~eq) & neg).sum(sum_dim).squeeze()
    tn = (eq & neg).sum(sum_dim).squeeze()
    return tp, fp, tn, fn


def _binary_stat_scores_update(
    preds: Tensor, target: Tensor, multidim_average: str = "global"
) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    """Stats from already-formatted label tensors ``[N, X]``."""
    return _samplewise_counts(preds, target, [0, 1] if multidim_average == "global" else [1])


def _binary_stats_fused(
    preds: Tensor, target: Tensor, threshold: float, ignore_index: Optional[int]
) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    """Global binary stats from *raw* inputs in one fused pass (format + count)."""
    buf = torch.zeros(4 + 6 + cls_ops.GRID_SLOTS, dtype=torch.long, device=target.device)
    states = tuple(buf[0:4])
    cls_ops.binary_stats_fused(preds, target, states, buf[4:], 1, threshold, ignore_index)
    return states


def _binary_stat_scores_compute(tp: Tensor, fp: Tensor, tn: Tensor, fn: Tensor, multidim_average: str = "global") -> Tensor:
    return torch.stack([tp, fp, tn, fn, tp + fn], dim=0 if multidim_average == "global" else 1).squeeze()


def binary_stat_scores(
    preds: Tensor,
    target: Tensor,
    threshold: float = 0.5,
    multidim_average: Literal["global", "samplewise"] = "global",
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """``[tp, fp, tn, fn, support]`` for binary tasks (``[N, 5]`` when ``multidim_average='samplewise'``)."""
    if validate_args:
        _binary_stat_scores_arg_validation(threshold, multidim_average, ignore_index)
        _binary_stat_scores_tensor_validation(preds, target, multidim_average, ignore_index)
    if multidim_average == "global":
        tp, fp, tn, fn = _binary_stats_fused(preds, target, threshold, ignore_index)
    else:
        preds, target = _binary_stat_scores_format(preds, target, threshold, ignore_index)
        tp, fp, tn, fn = _binary_stat_scores_update(preds, target, multidim_average)
    return _binary_stat_scores_compute(tp, fp, tn, fn, multidim_average)


# ---------------------------------------------------------------------------------------------------------
# multiclass
# ---------------------------------------------------------------------------------------------------------
def _multiclass_stat_scores_arg_validation(
    num_classes: int,
    top_k: int = 1,
    average: Optional[str] = "macro",
    multidim_average: str = "global",
    ignore_index: Optional[int] = None,
) -> None:
    if not isinstance(num_classes, int) or num_classes < 2:
        raise ValueError(f"Expected argument `num_classes` to be an integer larger than 1, but got {num_classes}")
    if not isinstance(top_k, int) and top_k < 1:
        raise ValueError(f"Expected argument `top_k` to be an integer larger than or equal to 1, but got {top_k}")
    if top_k > num_classes:
        raise ValueError(
            f"Expected argument `top_k` to be smaller or equal to `num_classes` but got {top_k} and {num_classes}"
        )
    _check_average(average)
    _check_mdmc(multidim_average)
    _check_ignore(ignore_index)


def _multiclass_stat_scores_tensor_validation(
    preds: Tensor,
    target: Tensor,
    num_classes: int,
    multidim_average: str = "global",
    ignore_index: Optional[int] = None,
    sink: Optional[DeferredChecks] = None,
    check_values: bool = True,
) -> None:
    if preds.ndim == target.ndim + 1:
        if not preds.is_floating_point():
            raise ValueError("If `preds` have one dimension more than `target`, `preds` should be a float tensor.")
        if preds.shape[1] != num_classes:
            raise ValueError(
                "If `preds` have one dimension more than `target`, `preds.shape[1]` should be"
                " equal to number of classes."
            )
        if preds.shape[2:] != target.shape[1:]:
            raise ValueError(
                "If `preds` have one dimension more than `target`, the shape of `preds` should be"
                " (N, C, ...), and the shape of `target` should be (N, ...)."
            )
        if multidim_average != "global" and preds.ndim < 3:
            raise ValueError(
                "If `preds` have one dimension more than `target`, the shape of `preds` should "
                " at least 3D when multidim_average is set to `samplewise`"
            )
    elif preds.ndim == target.ndim:
        if preds.shape != target.shape:
            raise ValueError(
                "The `preds` and `target` should have the same shape,",
                f" got `preds` with shape={preds.shape} and `target` with shape={target.shape}.",
            )
        if multidim_average != "global" and preds.ndim < 2:
            raise ValueError(
                "When `preds` and `target` have the same shape, the shape of `preds` should "
                " at least 2D when multidim_average is set to `samplewise`"
            )
    else:
        raise ValueError(
            "Either `preds` and `target` both should have the (same) shape (N, ...), or `target` should be (N, ...)"
            " and `preds` should be (N, C, ...)."
        )
    if not check_values:
        return
    if sink is None:
        n_unique = len(torch.unique(target))
        limit = num_classes if ignore_index is None else num_classes + 1
        if n_unique > limit:
            raise RuntimeError(
                "Detected more unique values in `target` than `num_classes`. Expected only"
                f" {limit} but found {n_unique} in `target`."
            )
        if not preds.is_floating_point():
            n_unique_p = len(torch.unique(preds))
            if n_unique_p > num_classes:
                raise RuntimeError(
                    "Detected more unique values in `preds` than `num_classes`. Expected only"
                    f" {num_classes} but found {n_unique_p} in `preds`."
                )
    else:
        # device-side range check (values must be valid class ids or the ignore index)
        bad_t = (target < 0) | (target >= num_classes)
        if ignore_index is not None:
            bad_t &= target != ignore_index
        sink.add(bad_t, RuntimeError, _TARGET_RANGE_MSG)
        if not preds.is_floating_point():
            sink.add((preds < 0) | (preds >= num_classes), RuntimeError, _PREDS_RANGE_MSG)


def _binary_value_flags(sink: Optional[DeferredChecks], preds: Tensor) -> Tuple[Optional[Tensor], Optional[Tensor]]:
    """Device flags for the fused binary / multilabel kernel: same keys as ``_check_binary_values`` records."""
    if sink is None:
        return None, None
    err_t = sink.flag(RuntimeError, "Detected values in `target` outside the allowed set.", preds.device)
    err_p = None if preds.is_floating_point() else sink.flag(
        RuntimeError, "Detected values in `preds` outside the allowed set.", preds.device
    )
    return err_t, err_p


_TARGET_RANGE_MSG = "Detected more unique values in `target` than `num_classes`."
_PREDS_RANGE_MSG = "Detected more unique values in `preds` than `num_classes`."


def _multiclass_range_flags(sink: Optional[DeferredChecks], preds: Tensor) -> Tuple[Optional[Tensor], Optional[Tensor]]:
    """Device flags the fused multiclass kernels OR into while streaming the batch (replaces the ~6 comparison /
    reduction kernels of the deferred value check)."""
    if sink is None:
        return None, None
    err_t = sink.flag(RuntimeError, _TARGET_RANGE_MSG, preds.device)
    err_p = None if preds.is_floating_point() else sink.flag(RuntimeError, _PREDS_RANGE_MSG, preds.device)
    return err_t, err_p


def _multiclass_pairs_view(preds: Tensor, target: Tensor, num_classes: int) -> Tuple[Tensor, Tensor]:
    """``[N, C, ...]`` scores -> ``[M, C]`` rows (or labels -> ``[M]``) and target -> ``[M]``."""
    if preds.ndim == target.ndim + 1:
        preds = torch.movedim(preds, 1, -1).reshape(-1, num_classes)
    else:
        preds = preds.reshape(-1)
        if preds.is_floating_point():
            preds = preds.long()
    return preds, target.reshape(-1)


def _multiclass_stat_scores_accumulate(
    preds: Tensor,
    target: Tensor,
    num_classes: int,
    states: Tuple[Tensor, Tensor, Tensor, Tensor],
    ticket: Tensor,
    ignore_index: Optional[int],
    micro: bool,
    err_t: Optional[Tensor] = None,
    err_p: Optional[Tensor] = None,
) -> None:
    """One fused pass (arg-max + per-class tp / fp / fn with tn derived) into ``states`` in place."""
    preds, target = _multiclass_pairs_view(preds, target, num_classes)
    cls_ops.mc_stat_scores_update(preds, target, num_classes, *states, ticket, ignore_index, micro, err_t, err_p)


def _multiclass_stat_scores_format(preds: Tensor, target: Tensor, top_k: int = 1) -> Tuple[Tensor, Tensor]:
    if preds.ndim == target.ndim + 1 and top_k == 1:
        preds = preds.argmax(dim=1)
    preds = preds.reshape(*preds.shape[:2], -1) if top_k != 1 else preds.reshape(preds.shape[0], -1)
    target = target.reshape(target.shape[0], -1)
    return preds, target


def _multiclass_onehot_stats(
    preds: Tensor,
    target: Tensor,
    num_classes: int,
    top_k: int,
    multidim_average: str,
    ignore_index: Optional[int],
) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    """Samplewise / top-k path: one-hot compare (reference stat_scores.py:363-393 semantics).

    GPU rows take ``csrc/rowwise.hip`` (k wave arg-max rounds per row, counts straight into the states): scores
    ``[N, C, X]`` are read as ``N * X`` rows of ``C``; label predictions ``[N, X]`` as ``N * X`` single picks."""
    if top_k > 1 and preds.ndim == 3 and cls_ops.row_kernel_ok(preds, num_classes):
        n, c, x = preds.shape
        rows = preds.movedim(1, -1).reshape(n * x, c) if x > 1 else preds.reshape(n, c)
        return cls_ops.topk_stats(rows, None, target, num_classes, top_k, ignore_index, n, multidim_average == "samplewise")
    if top_k == 1 and not preds.is_floating_point() and preds.shape == target.shape and ops.use_native(target):
        return cls_ops.topk_stats(None, preds, target, num_classes, 1, ignore_index, preds.shape[0], multidim_average == "samplewise")
    ignore_in =ignore_index is not None and 0 <= ignore_index <= num_classes - 1
    ignore_out = ignore_index is not None and not ignore_in
    if ignore_out:
        mask = target == ignore_index
        target = torch.where(mask, torch.full_like(target, num_classes), target)
        pmask = mask.unsqueeze(1).expand_as(preds) if preds.ndim > target.ndim else mask
        preds = torch.where(pmask, torch.full_like(preds, num_classes), preds)
    width = num_classes + 1 if ignore_out else num_classes
    if top_k > 1:
        preds_oh = torch.movedim(select_topk(preds, topk=top_k, dim=1), 1, -1)
    else:
        preds_oh = torch.nn.functional.one_hot(preds.long(), width)
    target_oh = torch.nn.functional.one_hot(target.long(), width)
    if ignore_index is not None:
        if ignore_in:
            target_oh[target == ignore_index, :] = -1
        else:
            preds_oh = preds_oh[..., :-1] if top_k == 1 else preds_oh
            target_oh = target_oh[..., :-1]
            target_oh[target == num_classes, :] = -1
    sum_dim = [0, 1] if multidim_average == "global" else [1]
    eq = target_oh == preds_oh
    tp = (eq & (target_oh == 1)).sum(sum_dim)
    fn = ((~eq) & (target_oh == 1)).sum(sum_dim)
    fp = ((~eq) & (target_oh == 0)).sum(sum_dim)
    tn = (eq & (target_oh == 0)).sum(sum_dim)
    return tp, fp, tn, fn


def _multiclass_stat_scores_update(
    preds: Tensor,
    target: Tensor,
    num_classes: int,
    top_k: int = 1,
    average: Optional[str] = "macro",
    multidim_average: str = "global",
    ignore_index: Optional[int] = None,
) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    """Stats from *raw* (unformatted) multiclass inputs."""
    if multidim_average == "samplewise" or top_k != 1:
        preds, target = _multiclass_stat_scores_format(preds, target, top_k)
        return _multiclass_onehot_stats(preds, target, num_classes, top_k, multidim_average, ignore_index)
    if ops.use_native(target):
        # one kernel, no [C, C] temporary (csrc/classification.hip mc_stat_scores_update)
        micro = average == "micro"
        width = 1 if micro else num_classes
        buf = torch.zeros(4 * width + cls_ops.GRID_SLOTS, dtype=torch.long, device=target.device)
        states = tuple(buf[0:4]) if micro else tuple(buf[: 4 * num_classes].view(4, num_classes))
        _multiclass_stat_scores_accumulate(preds, target, num_classes, states, buf[4 * width :], ignore_index, micro)
        return states
    if average == "micro":
        if preds.ndim == target.ndim + 1:
            preds = preds.argmax(dim=1)
        p, t = preds.reshape(-1), target.reshape(-1)
        if ignore_index is not None:
            keep = t != ignore_index
            n_valid = keep.sum()
            tp = ((p == t) & keep).sum()
            fp = ((p != t) & keep).sum()
        else:
            n_valid = torch.tensor(t.numel(), device=t.device)
            tp = (p == t).sum()
            fp = (p != t).sum()
        fn = fp.clone()
        tn = num_classes * n_valid - (fp + fn + tp)
        return tp, fp, tn, fn
    confmat = torch.zeros(num_classes, num_classes, dtype=torch.long, device=target.device)
    if preds.ndim == target.ndim + 1:
        # [N, C, ...] -> rows of C scores
        preds = torch.movedim(preds, 1, -1).reshape(-1, num_classes)
    cls_ops.mc_confmat_update(preds, target.reshape(-1), confmat, ignore_index)
    return _stats_from_confmat(confmat)


def _stats_from_confmat(confmat: Tensor) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    tp = confmat.diag()
    fp = confmat.sum(0) - tp
    fn = confmat.sum(1) - tp
    tn = confmat.sum() - (fp + fn + tp)
    return tp, fp, tn, fn


def _multiclass_stat_scores_compute(
    tp: Tensor, fp: Tensor, tn: Tensor, fn: Tensor, average: Optional[str] = "macro", multidim_average: str = "global"
) -> Tensor:
    res = torch.stack([tp, fp, tn, fn, tp + fn], dim=-1)
    sum_dim = 0 if multidim_average == "global" else 1
    if average == "micro":
        return res.sum(sum_dim) if res.ndim > 1 else res
    if average == "macro":
        return res.float().mean(sum_dim)
    if average == "weighted":
        weight = tp + fn
        if multidim_average == "global":
            return (res * (weight / weight.sum()).reshape(*weight.shape, 1)).sum(sum_dim)
        return (res * (weight / weight.sum(-1, keepdim=True)).reshape(*weight.shape, 1)).sum(sum_dim)
    if average is None or average == "none":
        return res
    return None


def multiclass_stat_scores(
    preds: Tensor,
    target: Tensor,
    num_classes: int,
    average: Optional[Literal["micro", "macro", "weighted", "none"]] = "macro",
    top_k: int = 1,
    multidim_average: Literal["global", "samplewise"] = "global",
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """``[tp, fp, tn, fn, support]`` for multiclass tasks (per class unless averaged)."""
    if validate_args:
        _multiclass_stat_scores_arg_validation(num_classes, top_k, average, multidim_average, ignore_index)
        _multiclass_stat_scores_tensor_validation(preds, target, num_classes, multidim_average, ignore_index)
    tp, fp, tn, fn = _multiclass_stat_scores_update(preds, target, num_classes, top_k, average, multidim_average, ignore_index)
    return _multiclass_stat_scores_compute(tp, fp, tn, fn, average, multidim_average)


# ---------------------------------------------------------------------------------------------------------
# multilabel
# ---------------------------------------------------------------------------------------------------------
def _multilabel_stat_scores_arg_validation(
    num_labels: int,
    threshold: float = 0.5,
    average: Optional[str] = "macro",
    multidim_average: str = "global",
    ignore_index: Optional[int] = None,
) -> None:
    if not isinstance(num_labels, int) or num_labels < 2:
        raise ValueError(f"Expected argument `num_labels` to be an integer larger than 1, but got {num_labels}")
    _check_threshold(threshold)
    _check_average(average)
    _check_mdmc(multidim_average)
    _check_ignore(ignore_index)


def _multilabel_stat_scores_tensor_validation(
    preds: Tensor,
    target: Tensor,
    num_labels: int,
    multidim_average: str,
    ignore_index: Optional[int] = None,
    sink: Optional[DeferredChecks] = None,
    check_values: bool = True,
) -> None:
    _check_same_shape(preds, target)
    if preds.shape[1] != num_labels:
        raise ValueError(
            "Expected both `target.shape[1]` and `preds.shape[1]` to be equal to the number of labels"
            f" but got {preds.shape[1]} and expected {num_labels}"
        )
    if check_values:
        _check_binary_values(target, "target", ignore_index, sink, label=False)
        if not preds.is_floating_point():
            _check_binary_values(preds, "preds", None, sink, label=True)
    if multidim_average != "global" and preds.ndim < 3:
        raise ValueError("Expected input to be at least 3D when multidim_average is set to `samplewise`")


def _multilabel_stat_scores_format(
    preds: Tensor, target: Tensor, num_labels: int, threshold: float = 0.5, ignore_index: Optional[int] = None
) -> Tuple[Tensor, Tensor]:
    if preds.is_floating_point():
        flag = cls_ops.range_flag(preds).bool()
        preds = torch.where(flag, preds.sigmoid(), preds) > threshold
    preds = preds.reshape(*preds.shape[:2], -1)
    target = target.reshape(*target.shape[:2], -1)
    if ignore_index is not None:
        target = torch.where(target == ignore_index, torch.full_like(target, -1), target)
    return preds, target


def _multilabel_stat_scores_update(
    preds: Tensor, target: Tensor, multidim_average: str = "global"
) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    return _samplewise_counts(preds, target, [0, -1] if multidim_average == "global" else [-1])


def _multilabel_stats_fused(
    preds: Tensor, target: Tensor, num_labels: int, threshold: float, ignore_index: Optional[int]
) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    buf = torch.zeros(10 * num_labels + cls_ops.GRID_SLOTS, dtype=torch.long, device=target.device)
    states = tuple(buf[: 4 * num_labels].view(4, num_labels))
    cls_ops.binary_stats_fused(preds, target, states, buf[4 * num_labels :], num_labels, threshold, ignore_index)
    return states


def _multilabel_stat_scores_compute(
    tp: Tensor, fp: Tensor, tn: Tensor, fn: Tensor, average: Optional[str] = "macro", multidim_average: str = "global"
) -> Tensor:
    res = torch.stack([tp, fp, tn, fn, tp + fn], dim=-1)
    sum_dim = 0 if multidim_average == "global" else 1
    if average == "micro":
        return res.sum(sum_dim)
    if average == "macro":
        return res.float().mean(sum_dim)
    if average == "weighted":
        w = tp + fn
        return (res * (w / w.sum()).reshape(*w.shape, 1)).sum(sum_dim)
    if average is None or average == "none":
        return res
    return None


def multilabel_stat_scores(
    preds: Tensor,
    target: Tensor,
    num_labels: int,
    threshold: float = 0.5,
    average: Optional[Literal["micro", "macro", "weighted", "none"]] = "macro",
    multidim_average: Literal["global", "samplewise"] = "global",
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """``[tp, fp, tn, fn, support]`` per label (or averaged) for multilabel tasks."""
    if validate_args:
        _multilabel_stat_scores_arg_validation(num_labels, threshold, average, multidim_average, ignore_index)
        _multilabel_stat_scores_tensor_validation(preds, target, num_labels, multidim_average, ignore_index)
    if multidim_average == "global":
        tp, fp, tn, fn = _multilabel_stats_fused(preds, target, num_labels, threshold, ignore_index)
    else:
        preds, target = _multilabel_stat_scores_format(preds, target, num_labels, threshold, ignore_index)
        tp, fp, tn, fn = _multilabel_stat_scores_update(preds, target, multidim_average)
    return _multilabel_stat_scores_compute(tp, fp, tn, fn, average, multidim_average)


# ---------------------------------------------------------------------------------------------------------
# task dispatch
# ---------------------------------------------------------------------------------------------------------
def stat_scores(
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
    task = ClassificationTask.from_str(task)
    assert multidim_average is not None  # noqa: S101
    if task == ClassificationTask.BINARY:
        return binary_stat_scores(preds, target, threshold, multidim_average, ignore_index, validate_args)
    if task == ClassificationTask.MULTICLASS:
        if not isinstance(num_classes, int):
            raise ValueError(f"`num_classes` is expected to be `int` but `{type(num_classes)} was passed.`")
        if not isinstance(top_k, int):
            raise ValueError(f"`top_k` is expected to be `int` but `{type(top_k)} was passed.`")
        return multiclass_stat_scores(preds, target, num_classes, average, top_k, multidim_average, ignore_index, validate_args)
    if task == ClassificationTask.MULTILABEL:
        if not isinstance(num_labels, int):
            raise ValueError(f"`num_labels` is expected to be `int` but `{type(num_labels)} was passed.`")
        return multilabel_stat_scores(preds, target, num_labels, threshold, average, multidim_average, ignore_index, validate_args)
    raise ValueError(f"Unsupported task `{task}`")
