"""SNR / SI-SNR / C-SI-SNR modules (API parity: reference ``audio/snr.py``; same state names)."""
from typing import Any

from torch import Tensor

from torchmetrics_forked_amd.audio._base import _MeanSignalMetric
from torchmetrics_forked_amd.functional.audio.snr import (
    complex_scale_invariant_signal_noise_ratio,
    scale_invariant_signal_noise_ratio,
    signal_noise_ratio,
)


class SignalNoiseRatio(_MeanSignalMetric):
    """Mean SNR over signals.

    Example:
        >>> import torch
        >>> from torchmetrics_forked_amd.audio import SignalNoiseRatio
        >>> SignalNoiseRatio()(torch.tensor([2.5, 0.0, 2.0, 8.0]), torch.tensor([3.0, -0.5, 2.0, 7.0]))
        tensor(16.1805)
    """

    _sum_name = "sum_snr"

    def __init__(self, zero_mean: bool = False, **kwargs: Any) -> None:
        super().__init__(**kwargs)
        self.zero_mean = zero_mean

    def _values(self, preds: Tensor, target: Tensor) -> Tensor:
        return signal_noise_ratio(preds=preds, target=target, zero_mean=self.zero_mean)


class ScaleInvariantSignalNoiseRatio(_MeanSignalMetric):
    """Mean SI-SNR over signals.

    Example:
        >>> import torch
        >>> from torchmetrics_forked_amd.audio import ScaleInvariantSignalNoiseRatio
        >>> preds = torch.tensor([2.5, 0.0, 2.0, 8.0, 4.2])
        >>> target = torch.tensor([3.0, 0.5, 2.0, 7.0, 4.0])
        >>> ScaleInvariantSignalNoiseRatio()(preds, target)
        tensor(20.6068)
    """

    _sum_name = "sum_si_snr"

    def _values(self, preds: Tensor, target: Tensor) -> Tensor:
        return scale_invariant_signal_noise_ratio(preds=preds, target=target)


class ComplexScaleInvariantSignalNoiseRatio(_MeanSignalMetric):
    """Mean complex SI-SNR over spectrograms."""

    is_differentiable = True
    _sum_name = "ci_snr_sum"
    _count_name = "num"

    def __init__(self, zero_mean: bool = False, **kwargs: Any) -> None:
        super().__init__(**kwargs)
        if not isinstance(zero_mean, bool):
            raise ValueError(f"Expected argument `zero_mean` to be an bool, but got {zero_mean}")
        self.zero_mean = zero_mean

    def _values(self, preds: Tensor, target: Tensor) -> Tensor:
        return complex_scale_invariant_signal_noise_ratio(preds=preds, target=target, zero_mean=self.zero_mean)
