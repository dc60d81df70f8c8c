"""Retrieval R-precision (API parity: reference ``functional/retrieval/r_precision.py:22-52``)."""
from torch import Tensor

from torchmetrics_forked_amd.functional.retrieval._grouped import Grouped, per_query_r_precision
from torchmetrics_forked_amd.utilities.checks import _check_retrieval_functional_inputs


def retrieval_r_precision(preds: Tensor, target: Tensor) -> Tensor:
    preds, target = _check_retrieval_functional_inputs(preds, target)
    return per_query_r_precision(Grouped(preds, target))[0]
