"""Cosine similarity (API parity: reference ``functional/regression/cosine_similarity.py:22-96``)."""
from typing import Optional, Tuple

import torch
from torch import Tensor

from torchmetrics_forked_amd.utilities.checks import _check_same_shape


def _cosine_similarity_update(preds: Tensor, target: Tensor) -> Tuple[Tensor, Tensor]:
    _check_same_shape(preds, target)
    return preds.float(), target.float()


def _cosine_similarity_compute(preds: Tensor, target: Tensor, reduction: Optional[str] = "sum") -> Tensor:
    dot = (preds * target).sum(dim=-1)
    sim = dot / (preds.norm(dim=-1) * target.norm(dim=-1))
    reductions = {"sum": torch.sum, "mean": torch.mean, "none": lambda x: x, None: lambda x: x}
    return reductions[reduction](sim)


def cosine_similarity(preds: Tensor, target: Tensor, reduction: Optional[str] = "sum") -> Tensor:
    return _cosine_similarity_compute(*_cosine_similarity_update(preds, target), reduction)
