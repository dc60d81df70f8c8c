"""Retrieval hit rate@k (API parity: reference ``functional/retrieval/hit_rate.py:22-58``)."""
from typing import Optional

from torch import Tensor

from torchmetrics_forked_amd.functional.retrieval._grouped import Grouped, per_query_hit_rate
from torchmetrics_forked_amd.utilities.checks import _check_retrieval_functional_inputs


def retrieval_hit_rate(preds: Tensor, target: Tensor, top_k: Optional[int] = None) -> Tensor:
    preds, target = _check_retrieval_functional_inputs(preds, target)
    if top_k is None:
        top_k = preds.shape[-1]
    if not (isinstance(top_k, int) and top_k > 0):
        raise ValueError("`top_k` has to be a positive integer or None")
    return per_query_hit_rate(Grouped(preds, target), top_k)[0]
