"""SpeechReverberationModulationEnergyRatio module (API parity: reference ``audio/srmr.py``); native filterbanks."""
from typing import Any, Optional

from torch import Tensor

from torchmetrics_forked_amd.audio._base import _MeanSignalMetric
from torchmetrics_forked_amd.functional.audio.srmr import _srmr_arg_validate, speech_reverberation_modulation_energy_ratio


class SpeechReverberationModulationEnergyRatio(_MeanSignalMetric):
    """Mean SRMR over signals (no target needed)."""

    is_differentiable = False  # deviation: the reference says True (torchaudio lfilter); the native IIR has no autograd
    _sum_name = "msum"

    def __init__(
        self,
        fs: int,
        n_cochlear_filters: int = 23,
        low_freq: float = 125,
        min_cf: float = 4,
        max_cf: Optional[float] = None,
        norm: bool = False,
        fast: bool = False,
        **kwargs: Any,
    ) -> None:
        super().__init__(**kwargs)
        _srmr_arg_validate(fs, n_cochlear_filters, low_freq, min_cf, max_cf, norm, fast)
        self.fs, self.n_cochlear_filters, self.low_freq = fs, n_cochlear_filters, low_freq
        self.min_cf, self.max_cf, self.norm, self.fast = min_cf, max_cf, norm, fast

    def update(self, preds: Tensor) -> None:  # type: ignore[override]
        v = speech_reverberation_modulation_energy_ratio(
            preds, self.fs, self.n_cochlear_filters, self.low_freq, self.min_cf, self.max_cf, self.norm, self.fast
        )
        self.msum += v.sum().to(self.msum.dtype)
        self.total += v.numel()
