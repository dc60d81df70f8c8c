"""Audio metrics (reference ``audio/__init__.py``)."""
from torchmetrics_forked_amd.audio.pesq import PerceptualEvaluationSpeechQuality
from torchmetrics_forked_amd.audio.pit import PermutationInvariantTraining
from torchmetrics_forked_amd.audio.sdr import (
    ScaleInvariantSignalDistortionRatio,
    SignalDistortionRatio,
    SourceAggregatedSignalDistortionRatio,
)
from torchmetrics_forked_amd.audio.snr import (
    ComplexScaleInvariantSignalNoiseRatio,
    ScaleInvariantSignalNoiseRatio,
    SignalNoiseRatio,
)
from torchmetrics_forked_amd.audio.srmr import SpeechReverberationModulationEnergyRatio
from torchmetrics_forked_amd.audio.stoi import ShortTimeObjectiveIntelligibility

__all__ = [
    "PermutationInvariantTraining",
    "ScaleInvariantSignalDistortionRatio",
    "SignalDistortionRatio",
    "SourceAggregatedSignalDistortionRatio",
    "ScaleInvariantSignalNoiseRatio",
    "SignalNoiseRatio",
    "ComplexScaleInvariantSignalNoiseRatio",
    "PerceptualEvaluationSpeechQuality",
    "ShortTimeObjectiveIntelligibility",
    "SpeechReverberationModulationEnergyRatio",
]
