"""ShortTimeObjectiveIntelligibility module (API parity: reference ``audio/stoi.py``); native STOI/ESTOI."""
from typing import Any

from torch import Tensor

from torchmetrics_forked_amd.audio._base import _MeanSignalMetric
from torchmetrics_forked_amd.functional.audio.stoi import short_time_objective_intelligibility


class ShortTimeObjectiveIntelligibility(_MeanSignalMetric):
    """Mean STOI (or ESTOI with ``extended=True``)."""

    is_differentiable = False
    _sum_name = "sum_stoi"

    def __init__(self, fs: int, extended: bool = False, **kwargs: Any) -> None:
        super().__init__(**kwargs)
        self.fs = fs
        self.extended = extended

    def _values(self, preds: Tensor, target: Tensor) -> Tensor:
        return short_time_objective_intelligibility(preds, target, self.fs, self.extended, keep_same_device=True)
