"""SQuAD module (API parity: reference ``text/squad.py``)."""
from typing import Any, Dict, Optional, Sequence, Union

import torch
from torch import Tensor

from torchmetrics_forked_amd.functional.text.squad import PREDS_TYPE, TARGETS_TYPE, _squad_compute, _squad_input_check, _squad_update
from torchmetrics_forked_amd.metric import Metric
from torchmetrics_forked_amd.utilities.plot import _AX_TYPE, _PLOT_OUT_TYPE


class SQuAD(Metric):
    """SQuAD v1.1 exact match and F1 (percent)."""

    is_differentiable: bool = False
    higher_is_better: bool = True
    full_state_update: bool = False
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 100.0
    f1_score: Tensor
    exact_match: Tensor
    total: Tensor

    def __init__(self, **kwargs: Any) -> None:
        super().__init__(**kwargs)
        self.add_state(name="f1_score", default=torch.tensor(0, dtype=torch.float), dist_reduce_fx="sum")
        self.add_state(name="exact_match", default=torch.tensor(0, dtype=torch.float), dist_reduce_fx="sum")
        self.add_state(name="total", default=torch.tensor(0, dtype=torch.int), dist_reduce_fx="sum")

    def update(self, preds: PREDS_TYPE, target: TARGETS_TYPE) -> None:
        preds_dict, target_dict = _squad_input_check(preds, target)
        f1, em, total = _squad_update(preds_dict, target_dict)
        self.f1_score += f1.to(self.f1_score)
        self.exact_match += em.to(self.exact_match)
        self.total += total.to(self.total)

    def compute(self) -> Dict[str, Tensor]:
        return _squad_compute(self.f1_score, self.exact_match, self.total)

    def plot(self, val: Optional[Union[Tensor, Sequence[Tensor]]] = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:
        return self._plot(val, ax)
