"""Mean-over-signals audio metric base: one ``sum`` state for the metric values and one for their count."""
from typing import Any, Callable, Dict, Optional, Sequence, Tuple, Union

from torch import Tensor, tensor

from torchmetrics_forked_amd.metric import Metric
from torchmetrics_forked_amd.utilities.plot import _AX_TYPE, _PLOT_OUT_TYPE


class _MeanSignalMetric(Metric):
    full_state_update: bool = False
    is_differentiable: bool = True
    higher_is_better: bool = True
    _sum_name: str = "sum_value"
    _count_name: str = "total"

    def __init__(self, **kwargs: Any) -> None:
        super().__init__(**kwargs)
        self.add_state(self._sum_name, default=tensor(0.0), dist_reduce_fx="sum")
        self.add_state(self._count_name, default=tensor(0), dist_reduce_fx="sum")

    def _values(self, preds: Tensor, target: Tensor) -> Tensor:
        raise NotImplementedError

    def update(self, preds: Tensor, target: Tensor) -> None:
        v = self._values(preds, target)
        acc, cnt = getattr(self, self._sum_name), getattr(self, self._count_name)
        acc += v.sum().to(acc.dtype)  # in place: the state keeps its dtype (as the reference's ``+=``)
        cnt += v.numel()

    def compute(self) -> Tensor:
        return getattr(self, self._sum_name) / getattr(self, self._count_name)

    def plot(self, val: Optional[Union[Tensor, Sequence[Tensor]]] = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:
        return self._plot(val, ax)
