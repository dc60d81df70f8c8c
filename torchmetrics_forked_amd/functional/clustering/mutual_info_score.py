"""Mutual information (API parity: reference ``functional/clustering/mutual_info_score.py:21-80``)."""
import torch
from torch import Tensor

from torchmetrics_forked_amd.functional.clustering.utils import calculate_contingency_matrix, check_cluster_labels


def _mutual_info_score_update(preds: Tensor, target: Tensor) -> Tensor:
    check_cluster_labels(preds, target)
    return calculate_contingency_matrix(preds, target)


def _mutual_info_score_compute(contingency: Tensor) -> Tensor:
    n = contingency.sum()
    u, v = contingency.sum(dim=1), contingency.sum(dim=0)
    nzu, nzv = torch.nonzero(contingency, as_tuple=True)
    nij = contingency[nzu, nzv]
    log_outer = torch.log(u[nzu]) + torch.log(v[nzv])
    return (nij / n * (torch.log(n) + torch.log(nij) - log_outer)).sum()


def mutual_info_score(preds: Tensor, target: Tensor) -> Tensor:
    return _mutual_info_score_compute(_mutual_info_score_update(preds, target))
