"""Retrieval metrics (API parity: reference ``retrieval/{average_precision,reciprocal_rank,precision,recall,
fall_out,hit_rate,r_precision,ndcg}.py``)."""
from typing import Any, Optional

from torch import Tensor

from torchmetrics_forked_amd.functional.retrieval import _grouped as G
from torchmetrics_forked_amd.retrieval.base import RetrievalMetric


def _check_top_k(top_k: Optional[int]) -> None:
    if top_k is not None and not (isinstance(top_k, int) and top_k > 0):
        raise ValueError("`top_k` has to be a positive integer or None")


class _Bounded(RetrievalMetric):
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0


class RetrievalMAP(_Bounded):
    """Mean average precision over queries.

    Example:
        >>> import torch
        >>> from torchmetrics_forked_amd.retrieval import RetrievalMAP
        >>> indexes = torch.tensor([0, 0, 0, 1, 1, 1, 1])
        >>> preds = torch.tensor([0.2, 0.3, 0.5, 0.1, 0.3, 0.5, 0.2])
        >>> target = torch.tensor([False, False, True, False, True, False, True])
        >>> RetrievalMAP()(preds, target, indexes=indexes)
        tensor(0.7917)
    """
    def __init__(self, empty_target_action: str = "neg", ignore_index: Optional[int] = None, top_k: Optional[int] = None, **kwargs: Any) -> None:
        super().__init__(empty_target_action=empty_target_action, ignore_index=ignore_index, **kwargs)
        if top_k is not None and not isinstance(top_k, int) and top_k <= 0:
            raise ValueError(f"Argument ``top_k`` has to be a positive integer or None, but got {top_k}")
        self.k = top_k

    def _per_query(self, g: G.Grouped) -> Tensor:
        return G.per_query_average_precision(g, self.k)


class RetrievalMRR(_Bounded):
    """Mean reciprocal rank over queries.

    Example:
        >>> import torch
        >>> from torchmetrics_forked_amd.retrieval import RetrievalMRR
        >>> indexes = torch.tensor([0, 0, 0, 1, 1, 1, 1])
        >>> preds = torch.tensor([0.2, 0.3, 0.5, 0.1, 0.3, 0.5, 0.2])
        >>> target = torch.tensor([False, False, True, False, True, False, True])
        >>> RetrievalMRR()(preds, target, indexes=indexes)
        tensor(0.7500)
    """
    def __init__(self, empty_target_action: str = "neg", ignore_index: Optional[int] = None, top_k: Optional[int] = None, **kwargs: Any) -> None:
        super().__init__(empty_target_action=empty_target_action, ignore_index=ignore_index, **kwargs)
        if top_k is not None and not isinstance(top_k, int) and top_k <= 0:
            raise ValueError(f"Argument ``top_k`` has to be a positive integer or None, but got {top_k}")
        self.top_k = top_k

    def _per_query(self, g: G.Grouped) -> Tensor:
        return G.per_query_reciprocal_rank(g, self.top_k)


class RetrievalPrecision(_Bounded):
    """RetrievalPrecision over queries.

    Example:
        >>> import torch
        >>> from torchmetrics_forked_amd.retrieval import RetrievalPrecision
        >>> indexes = torch.tensor([0, 0, 0, 1, 1, 1, 1])
        >>> preds = torch.tensor([0.2, 0.3, 0.5, 0.1, 0.3, 0.5, 0.2])
        >>> target = torch.tensor([False, False, True, False, True, False, True])
        >>> RetrievalPrecision(top_k=2)(preds, target, indexes=indexes)
        tensor(0.5000)
    """
    def __init__(
        self,
        empty_target_action: str = "neg",
        ignore_index: Optional[int] = None,
        top_k: Optional[int] = None,
        adaptive_k: bool = False,
        **kwargs: Any,
    ) -> None:
        super().__init__(empty_target_action=empty_target_action, ignore_index=ignore_index, **kwargs)
        _check_top_k(top_k)
        if not isinstance(adaptive_k, bool):
            raise ValueError("`adaptive_k` has to be a boolean")
        self.top_k = top_k
        self.adaptive_k = adaptive_k

    def _per_query(self, g: G.Grouped) -> Tensor:
        return G.per_query_precision(g, self.top_k, self.adaptive_k)


class RetrievalRecall(_Bounded):
    """RetrievalRecall over queries.

    Example:
        >>> import torch
        >>> from torchmetrics_forked_amd.retrieval import RetrievalRecall
        >>> indexes = torch.tensor([0, 0, 0, 1, 1, 1, 1])
        >>> preds = torch.tensor([0.2, 0.3, 0.5, 0.1, 0.3, 0.5, 0.2])
        >>> target = torch.tensor([False, False, True, False, True, False, True])
        >>> RetrievalRecall(top_k=2)(preds, target, indexes=indexes)
        tensor(0.7500)
    """
    def __init__(self, empty_target_action: str = "neg", ignore_index: Optional[int] = None, top_k: Optional[int] = None, **kwargs: Any) -> None:
        super().__init__(empty_target_action=empty_target_action, ignore_index=ignore_index, **kwargs)
        _check_top_k(top_k)
        self.top_k = top_k

    def _per_query(self, g: G.Grouped) -> Tensor:
        return G.per_query_recall(g, self.top_k)


class RetrievalFallOut(_Bounded):
    """RetrievalFallOut over queries.

    Example:
        >>> import torch
        >>> from torchmetrics_forked_amd.retrieval import RetrievalFallOut
        >>> indexes = torch.tensor([0, 0, 0, 1, 1, 1, 1])
        >>> preds = torch.tensor([0.2, 0.3, 0.5, 0.1, 0.3, 0.5, 0.2])
        >>> target = torch.tensor([False, False, True, False, True, False, True])
        >>> RetrievalFallOut(top_k=2)(preds, target, indexes=indexes)
        tensor(0.5000)
    """
    higher_is_better: bool = False
    _empty_on_negatives = True

    def __init__(self, empty_target_action: str = "pos", ignore_index: Optional[int] = None, top_k: Optional[int] = None, **kwargs: Any) -> None:
        super().__init__(empty_target_action=empty_target_action, ignore_index=ignore_index, **kwargs)
        _check_top_k(top_k)
        self.top_k = top_k

    def _per_query(self, g: G.Grouped) -> Tensor:
        return G.per_query_fall_out(g, self.top_k)


class RetrievalHitRate(_Bounded):
    """RetrievalHitRate over queries.

    Example:
        >>> import torch
        >>> from torchmetrics_forked_amd.retrieval import RetrievalHitRate
        >>> indexes = torch.tensor([0, 0, 0, 1, 1, 1, 1])
        >>> preds = torch.tensor([0.2, 0.3, 0.5, 0.1, 0.3, 0.5, 0.2])
        >>> target = torch.tensor([False, False, True, False, True, False, True])
        >>> RetrievalHitRate(top_k=2)(preds, target, indexes=indexes)
        tensor(1.)
    """
    def __init__(self, empty_target_action: str = "neg", ignore_index: Optional[int] = None, top_k: Optional[int] = None, **kwargs: Any) -> None:
        super().__init__(empty_target_action=empty_target_action, ignore_index=ignore_index, **kwargs)
        _check_top_k(top_k)
        self.top_k = top_k

    def _per_query(self, g: G.Grouped) -> Tensor:
        return G.per_query_hit_rate(g, self.top_k)


class RetrievalRPrecision(_Bounded):
    """RetrievalRPrecision over queries.

    Example:
        >>> import torch
        >>> from torchmetrics_forked_amd.retrieval import RetrievalRPrecision
        >>> indexes = torch.tensor([0, 0, 0, 1, 1, 1, 1])
        >>> preds = torch.tensor([0.2, 0.3, 0.5, 0.1, 0.3, 0.5, 0.2])
        >>> target = torch.tensor([False, False, True, False, True, False, True])
        >>> RetrievalRPrecision()(preds, target, indexes=indexes)
        tensor(0.7500)
    """
    def _per_query(self, g: G.Grouped) -> Tensor:
        return G.per_query_r_precision(g)


class RetrievalNormalizedDCG(_Bounded):
    """Normalized discounted cumulative gain over queries.

    Example:
        >>> import torch
        >>> from torchmetrics_forked_amd.retrieval import RetrievalNormalizedDCG
        >>> indexes = torch.tensor([0, 0, 0, 1, 1, 1, 1])
        >>> preds = torch.tensor([0.2, 0.3, 0.5, 0.1, 0.3, 0.5, 0.2])
        >>> target = torch.tensor([0, 0, 2, 0, 1, 0, 3])
        >>> RetrievalNormalizedDCG()(preds, target, indexes=indexes)
        tensor(0.7934)
    """
    def __init__(self, empty_target_action: str = "neg", ignore_index: Optional[int] = None, top_k: Optional[int] = None, **kwargs: Any) -> None:
        super().__init__(empty_target_action=empty_target_action, ignore_index=ignore_index, **kwargs)
        _check_top_k(top_k)
        self.top_k = top_k
        self.allow_non_binary_target = True

    def _per_query(self, g: G.Grouped) -> Tensor:
        return G.per_query_ndcg(g, self.top_k)
