"""Rand score (API parity: reference ``functional/clustering/rand_score.py``)."""
import torch
from torch import Tensor

from torchmetrics_forked_amd.functional.clustering.utils import (
    calculate_contingency_matrix,
    calculate_pair_cluster_confusion_matrix,
    check_cluster_labels,
)


def _rand_score_update(preds: Tensor, target: Tensor) -> Tensor:
    check_cluster_labels(preds, target)
    return calculate_contingency_matrix(preds, target)


def _rand_score_compute(contingency: Tensor) -> Tensor:
    pair = calculate_pair_cluster_confusion_matrix(contingency=contingency)
    num, den = pair.diagonal().sum(), pair.sum()
    if num == den or den == 0:
        return torch.ones_like(num, dtype=torch.float32)
    return num / den


def rand_score(preds: Tensor, target: Tensor) -> Tensor:
    return _rand_score_compute(_rand_score_update(preds, target))
