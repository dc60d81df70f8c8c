"""Deprecated root-import shims for ``audio`` (reference ``audio/_deprecated.py``)."""
from torchmetrics_forked_amd.audio import (
    PermutationInvariantTraining,
    ScaleInvariantSignalDistortionRatio,
    ScaleInvariantSignalNoiseRatio,
    SignalDistortionRatio,
    SignalNoiseRatio,
)
from torchmetrics_forked_amd.utilities.deprecation import deprecated_class

_PermutationInvariantTraining = deprecated_class(PermutationInvariantTraining, "audio")
_ScaleInvariantSignalDistortionRatio = deprecated_class(ScaleInvariantSignalDistortionRatio, "audio")
_ScaleInvariantSignalNoiseRatio = deprecated_class(ScaleInvariantSignalNoiseRatio, "audio")
_SignalDistortionRatio = deprecated_class(SignalDistortionRatio, "audio")
_SignalNoiseRatio = deprecated_class(SignalNoiseRatio, "audio")
