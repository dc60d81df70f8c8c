"""Multilabel ranking metrics (API parity: reference ``functional/classification/ranking.py:27-268``).

The reference scores label-ranking average precision with a Python loop over samples (two ``torch.unique`` calls
per row).  Here every row is ranked at once: ``rank_j = #{k : p_k >= p_j}`` (the reference's max-rank tie rule)
via one batched ``sort`` + ``searchsorted``; the within-relevant rank uses the same search on a copy whose
non-relevant entries are pushed to ``+inf``.
"""
from typing import Any, Optional, Tuple

import torch
from torch import Tensor

from torchmetrics_forked_amd.functional.classification._formats import multilabel_format
from torchmetrics_forked_amd.functional.classification.confusion_matrix import _multilabel_confusion_matrix_arg_validation
from torchmetrics_forked_amd.functional.classification.stat_scores import _multilabel_stat_scores_tensor_validation
from torchmetrics_forked_amd.ops import classification as cls_ops


def _rank_data(x: Tensor) -> Tensor:
    """Max-rank of every element (ties share the highest rank), reference ``ranking.py:27``."""
    _, inverse, counts = torch.unique(x, sorted=True, return_inverse=True, return_counts=True)
    return torch.cumsum(counts, 0)[inverse]


def _ranking_reduce(score: Tensor, num_elements: int) -> Tensor:
    return score / num_elements


def _multilabel_ranking_tensor_validation(
    preds: Tensor, target: Tensor, num_labels: int, ignore_index: Optional[int] = None, sink: Optional[Any] = None
) -> None:
    _multilabel_stat_scores_tensor_validation(preds, target, num_labels, "global", ignore_index, sink)
    if not preds.is_floating_point():
        raise ValueError(f"Expected preds tensor to be floating point, but received input with dtype {preds.dtype}")


def _ranking_format(preds: Tensor, target: Tensor, num_labels: int, ignore_index: Optional[int]) -> Tuple[Tensor, Tensor]:
    return multilabel_format(preds, target, num_labels, threshold=0.0, ignore_index=ignore_index, should_threshold=False)


def _multilabel_coverage_error_update(preds: Tensor, target: Tensor) -> Tuple[Tensor, int]:
    if cls_ops.row_kernel_ok(preds, preds.shape[-1]) and preds.ndim == 2:
        out, _ = cls_ops.ml_ranking(preds, target, 0)  # csrc/rowwise.hip, one wave per row
        return out.sum(), out.numel()
    offset = torch.where(target == 0, preds.min().abs() + 10, torch.zeros((), dtype=preds.dtype, device=preds.device))
    preds_min = (preds + offset).min(dim=1).values
    coverage = (preds >= preds_min[:, None]).sum(dim=1).to(torch.float32)
    return coverage.sum(), coverage.numel()


def _row_max_rank(values: Tensor, queries: Tensor) -> Tensor:
    """For each row: number of ``values`` entries <= each query (batched)."""
    srt = values.sort(dim=1).values.contiguous()
    return torch.searchsorted(srt, queries.contiguous(), right=True)


def _multilabel_ranking_average_precision_update(preds: Tensor, target: Tensor) -> Tuple[Tensor, int]:
    num_preds, num_labels = preds.shape
    if num_preds == 0:
        return torch.tensor(0.0, device=preds.device), 0
    if cls_ops.row_kernel_ok(preds, num_labels):
        out, _ = cls_ops.ml_ranking(preds, target, 1)
        return out.sum(), num_preds
    neg = -preds.float()
    relevant = target == 1
    n_rel = relevant.sum(1)
    rank_all = _row_max_rank(neg, neg).float()
    neg_rel = torch.where(relevant, neg, torch.full_like(neg, float("inf")))
    rank_rel = _row_max_rank(neg_rel, neg).float()
    ratio = torch.where(relevant, rank_rel / rank_all, torch.zeros_like(rank_all))
    per_row = ratio.sum(1) / n_rel.clamp(min=1)
    degenerate = (n_rel == 0) | (n_rel == num_labels)
    per_row = torch.where(degenerate, torch.ones_like(per_row), per_row)
    return per_row.sum(), num_preds


def _multilabel_ranking_loss_update(preds: Tensor, target: Tensor) -> Tuple[Tensor, Tensor]:
    """Reference semantics (rows with no or only relevant labels are dropped; an all-degenerate batch counts as
    loss 0 over 1 sample) computed with masks instead of boolean indexing, so the GPU update never waits on the
    host for the number of kept rows."""
    num_preds, num_labels = preds.shape
    if num_preds and cls_ops.row_kernel_ok(preds, num_labels):
        out, flag = cls_ops.ml_ranking(preds, target, 2)
        one = torch.ones((), dtype=torch.long, device=preds.device)
        return out.sum(), torch.where(flag[0] != 0, one * num_preds, one)
    relevant = target == 1
    num_relevant = relevant.sum(dim=1)
    mask = (num_relevant > 0) & (num_relevant < num_labels)
    inverse = preds.argsort(dim=1, stable=True).argsort(dim=1, stable=True)
    per_label_loss = ((num_labels - inverse) * relevant).to(torch.float32)
    correction = 0.5 * num_relevant * (num_relevant + 1)
    denom = (num_relevant * (num_labels - num_relevant)).clamp(min=1)
    loss = torch.where(mask, (per_label_loss.sum(dim=1) - correction) / denom, torch.zeros((), device=preds.device))
    n = torch.where(mask.any(), torch.full((), num_preds, device=preds.device), torch.ones((), dtype=torch.long, device=preds.device))
    return loss.sum(), n


def _validate(preds: Tensor, target: Tensor, num_labels: int, ignore_index: Optional[int]) -> None:
    _multilabel_confusion_matrix_arg_validation(num_labels, threshold=0.0, ignore_index=ignore_index)
    _multilabel_ranking_tensor_validation(preds, target, num_labels, ignore_index)


def multilabel_coverage_error(
    preds: Tensor, target: Tensor, num_labels: int, ignore_index: Optional[int] = None, validate_args: bool = True
) -> Tensor:
    if validate_args:
        _validate(preds, target, num_labels, ignore_index)
    preds, target = _ranking_format(preds, target, num_labels, ignore_index)
    return _ranking_reduce(*_multilabel_coverage_error_update(preds, target))


def multilabel_ranking_average_precision(
    preds: Tensor, target: Tensor, num_labels: int, ignore_index: Optional[int] = None, validate_args: bool = True
) -> Tensor:
    if validate_args:
        _validate(preds, target, num_labels, ignore_index)
    preds, target = _ranking_format(preds, target, num_labels, ignore_index)
    return _ranking_reduce(*_multilabel_ranking_average_precision_update(preds, target))


def multilabel_ranking_loss(
    preds: Tensor, target: Tensor, num_labels: int, ignore_index: Optional[int] = None, validate_args: bool = True
) -> Tensor:
    if validate_args:
        _validate(preds, target, num_labels, ignore_index)
    preds, target = _ranking_format(preds, target, num_labels, ignore_index)
    return _ranking_reduce(*_multilabel_ranking_loss_update(preds, target))
