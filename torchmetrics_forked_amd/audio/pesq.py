"""PerceptualEvaluationSpeechQuality module (API parity: reference ``audio/pesq.py``; requires ``pesq``)."""
from typing import Any

from torch import Tensor

from torchmetrics_forked_amd.audio._base import _MeanSignalMetric
from torchmetrics_forked_amd.functional.audio.pesq import _PESQ_AVAILABLE, perceptual_evaluation_speech_quality


class PerceptualEvaluationSpeechQuality(_MeanSignalMetric):
    """Mean PESQ (ITU-T P.862) through the ``pesq`` package."""

    is_differentiable = False
    _sum_name = "sum_pesq"

    def __init__(self, fs: int, mode: str, n_processes: int = 1, **kwargs: Any) -> None:
        super().__init__(**kwargs)
        if not _PESQ_AVAILABLE:
            raise ModuleNotFoundError("PerceptualEvaluationSpeechQuality metric requires that `pesq` is installed.")
        if fs not in (8000, 16000):
            raise ValueError(f"Expected argument `fs` to either be 8000 or 16000 but got {fs}")
        self.fs = fs
        if mode not in ("wb", "nb"):
            raise ValueError(f"Expected argument `mode` to either be 'wb' or 'nb' but got {mode}")
        self.mode = mode
        if not isinstance(n_processes, int) or n_processes <= 0:
            raise ValueError(f"Expected argument `n_processes` to be an int larger than 0 but got {n_processes}")
        self.n_processes = n_processes

    def _values(self, preds: Tensor, target: Tensor) -> Tensor:
        return perceptual_evaluation_speech_quality(preds, target, self.fs, self.mode, True, self.n_processes)
