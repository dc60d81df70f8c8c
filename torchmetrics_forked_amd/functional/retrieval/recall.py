"""Retrieval recall@k (API parity: reference ``functional/retrieval/recall.py:22-62``)."""
from typing import Optional

from torch import Tensor

from torchmetrics_forked_amd.functional.retrieval._grouped import Grouped, per_query_recall
from torchmetrics_forked_amd.utilities.checks import _check_retrieval_functional_inputs


def retrieval_recall(preds: Tensor, target: Tensor, top_k: Optional[int] = None) -> Tensor:
    preds, target = _check_retrieval_functional_inputs(preds, target)
    if top_k is None:
        top_k = preds.shape[-1]
    if not (isinstance(top_k, int) and top_k > 0):
        raise ValueError("`top_k` has to be a positive integer or None")
    return per_query_recall(Grouped(preds, target), top_k)[0]
