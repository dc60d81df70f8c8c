"""Shared pieces of the regression modules."""
from typing import Any, Optional, Sequence, Union

from torch import Tensor

from torchmetrics_forked_amd.metric import Metric
from torchmetrics_forked_amd.utilities.plot import _AX_TYPE, _PLOT_OUT_TYPE


class _RegressionMetric(Metric):
    is_differentiable: bool = True
    full_state_update: bool = False

    def plot(self, val: Optional[Union[Tensor, Sequence[Tensor]]] = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:
        return self._plot(val, ax)
