"""Retrieval precision-recall curve over k and recall at fixed precision (API parity: reference
``retrieval/precision_recall_curve.py:32-330``)."""
from typing import Any, Optional, Sequence, Tuple, Union

import torch
from torch import Tensor

from torchmetrics_forked_amd.functional.retrieval import _grouped as G
from torchmetrics_forked_amd.metric import Metric
from torchmetrics_forked_amd.retrieval.base import RetrievalMetric
from torchmetrics_forked_amd.utilities.data import dim_zero_cat
from torchmetrics_forked_amd.utilities.plot import _AX_TYPE, _PLOT_OUT_TYPE, plot_curve


def _retrieval_recall_at_fixed_precision(
    precision: Tensor, recall: Tensor, top_k: Tensor, min_precision: float
) -> Tuple[Tensor, Tensor]:
    """Largest recall (ties -> largest k) among cut-offs whose precision reaches ``min_precision``."""
    ok = precision >= min_precision
    if bool(ok.any()):
        r, k = recall[ok], top_k[ok]
        best = r.max()
        max_recall, best_k = best, k[r == best].max()
    else:
        max_recall = torch.tensor(0.0, device=recall.device, dtype=recall.dtype)
        best_k = torch.tensor(len(top_k))
    if max_recall == 0.0:
        best_k = torch.tensor(len(top_k), device=top_k.device, dtype=top_k.dtype)
    return max_recall, best_k


class RetrievalPrecisionRecallCurve(RetrievalMetric):
    is_differentiable: bool = False
    higher_is_better: bool = True
    full_state_update: bool = False

    def __init__(
        self,
        max_k: Optional[int] = None,
        adaptive_k: bool = False,
        empty_target_action: str = "neg",
        ignore_index: Optional[int] = None,
        **kwargs: Any,
    ) -> None:
        super().__init__(empty_target_action=empty_target_action, ignore_index=ignore_index, **kwargs)
        if max_k is not None and not (isinstance(max_k, int) and max_k > 0):
            raise ValueError("`max_k` has to be a positive integer or None")
        self.max_k = max_k
        if not isinstance(adaptive_k, bool):
            raise ValueError("`adaptive_k` has to be a boolean")
        self.adaptive_k = adaptive_k

    def compute(self) -> Tuple[Tensor, Tensor, Tensor]:
        preds = dim_zero_cat(self.preds)
        g = self._grouped()
        if self.max_k is not None:
            max_k = self.max_k
        elif self._sharded_active:  # the longest query over all ranks
            from torchmetrics_forked_amd.parallel.shard import all_reduce_max

            local = g.sizes.max().reshape(1) if g.sizes.numel() else torch.zeros(1, dtype=torch.long, device=preds.device)
            max_k = int(all_reduce_max(local.long(), self._shard_group))
        else:
            max_k = int(g.sizes.max())
        precision, recall, _ = G.per_query_pr_curve(g, max_k, self.adaptive_k)
        empty = self._empty_queries(g)
        if self._sharded_active:
            return (self._sharded_mean(precision.to(preds), empty, preds.dtype, (max_k,)),
                    self._sharded_mean(recall.to(preds), empty, preds.dtype, (max_k,)),
                    torch.arange(1, max_k + 1, device=preds.device))
        precision = self._apply_empty_action(precision, empty, (max_k,))
        recall = self._apply_empty_action(recall, empty, (max_k,))
        if precision.shape[0]:
            precision, recall = precision.to(preds).mean(0), recall.to(preds).mean(0)
        else:
            precision, recall = torch.zeros(max_k).to(preds), torch.zeros(max_k).to(preds)
        return precision, recall, torch.arange(1, max_k + 1, device=preds.device)

    def plot(self, curve: Optional[Tuple[Tensor, Tensor, Tensor]] = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:
        curve = curve or self.compute()
        return plot_curve(curve, ax=ax, label_names=("False positive rate", "True positive rate"), name=self.__class__.__name__)


class RetrievalRecallAtFixedPrecision(RetrievalPrecisionRecallCurve):
    higher_is_better = True

    def __init__(
        self,
        min_precision: float = 0.0,
        max_k: Optional[int] = None,
        adaptive_k: bool = False,
        empty_target_action: str = "neg",
        ignore_index: Optional[int] = None,
        **kwargs: Any,
    ) -> None:
        super().__init__(max_k=max_k, adaptive_k=adaptive_k, empty_target_action=empty_target_action, ignore_index=ignore_index, **kwargs)
        if not (isinstance(min_precision, float) and 0.0 <= min_precision <= 1.0):
            raise ValueError("`min_precision` has to be a positive float between 0 and 1")
        self.min_precision = min_precision

    def compute(self) -> Tuple[Tensor, Tensor]:  # type: ignore[override]
        precisions, recalls, top_k = super().compute()
        return _retrieval_recall_at_fixed_precision(precisions, recalls, top_k, self.min_precision)

    def plot(self, val: Optional[Union[Tensor, Sequence[Tensor]]] = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:  # type: ignore[override]
        val = val if val is not None else self.compute()[0]
        return self._plot(val, ax)
