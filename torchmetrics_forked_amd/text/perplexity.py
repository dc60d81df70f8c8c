"""Perplexity module (API parity: reference ``text/perplexity.py``); fused token-NLL kernel on GPU."""
from typing import Any, Dict, Optional, Sequence, Union

from torch import Tensor, tensor

from torchmetrics_forked_amd.functional.text.perplexity import _perplexity_compute, _perplexity_update
from torchmetrics_forked_amd.metric import Metric
from torchmetrics_forked_amd.utilities.plot import _AX_TYPE, _PLOT_OUT_TYPE


class Perplexity(Metric):
    """exp(mean negative log-likelihood of the target tokens)."""

    is_differentiable = True
    higher_is_better = False
    full_state_update = False
    plot_lower_bound: float = 0.0
    total_log_probs: Tensor
    count: Tensor

    def __init__(self, ignore_index: Optional[int] = None, **kwargs: Dict[str, Any]) -> None:
        super().__init__(**kwargs)
        if ignore_index is not None and not isinstance(ignore_index, int):
            raise ValueError(f"Argument `ignore_index` expected to either be `None` or an `int` but got {ignore_index}")
        self.ignore_index = ignore_index
        self.add_state("total_log_probs", default=tensor(0.0), dist_reduce_fx="sum")
        self.add_state("count", default=tensor(0.0), dist_reduce_fx="sum")

    def update(self, preds: Tensor, target: Tensor) -> None:
        total, count = _perplexity_update(preds, target, self.ignore_index)
        self.total_log_probs = self.total_log_probs + total.to(self.total_log_probs.dtype)
        self.count = self.count + count

    def compute(self) -> Tensor:
        return _perplexity_compute(self.total_log_probs, self.count)

    def plot(self, val: Optional[Union[Tensor, Sequence[Tensor]]] = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:
        return self._plot(val, ax)
