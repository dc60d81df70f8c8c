"""Fowlkes-Mallows index (API parity: reference ``functional/clustering/fowlkes_mallows_index.py``)."""
from typing import Tuple

import torch
from torch import Tensor, tensor

from torchmetrics_forked_amd.functional.clustering.utils import calculate_contingency_matrix, check_cluster_labels


def _fowlkes_mallows_index_update(preds: Tensor, target: Tensor) -> Tuple[Tensor, int]:
    check_cluster_labels(preds, target)
    return calculate_contingency_matrix(preds, target), preds.size(0)


def _fowlkes_mallows_index_compute(contingency: Tensor, n: int) -> Tensor:
    tk = torch.sum(contingency**2) - n
    if torch.allclose(tk, tensor(0, device=tk.device)):
        return torch.tensor(0.0, device=contingency.device)
    pk = torch.sum(contingency.sum(dim=0) ** 2) - n
    qk = torch.sum(contingency.sum(dim=1) ** 2) - n
    return torch.sqrt(tk / pk) * torch.sqrt(tk / qk)


def fowlkes_mallows_index(preds: Tensor, target: Tensor) -> Tensor:
    return _fowlkes_mallows_index_compute(*_fowlkes_mallows_index_update(preds, target))
