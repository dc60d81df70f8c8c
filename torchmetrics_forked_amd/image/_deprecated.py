"""Deprecated root-import shims for ``image`` (reference ``image/_deprecated.py``)."""
from torchmetrics_forked_amd.image import (
    ErrorRelativeGlobalDimensionlessSynthesis,
    MultiScaleStructuralSimilarityIndexMeasure,
    PeakSignalNoiseRatio,
    RelativeAverageSpectralError,
    RootMeanSquaredErrorUsingSlidingWindow,
    SpectralAngleMapper,
    SpectralDistortionIndex,
    StructuralSimilarityIndexMeasure,
    TotalVariation,
    UniversalImageQualityIndex,
)
from torchmetrics_forked_amd.utilities.deprecation import deprecated_class

_ErrorRelativeGlobalDimensionlessSynthesis = deprecated_class(ErrorRelativeGlobalDimensionlessSynthesis, "image")
_MultiScaleStructuralSimilarityIndexMeasure = deprecated_class(MultiScaleStructuralSimilarityIndexMeasure, "image")
_PeakSignalNoiseRatio = deprecated_class(PeakSignalNoiseRatio, "image")
_RelativeAverageSpectralError = deprecated_class(RelativeAverageSpectralError, "image")
_RootMeanSquaredErrorUsingSlidingWindow = deprecated_class(RootMeanSquaredErrorUsingSlidingWindow, "image")
_SpectralAngleMapper = deprecated_class(SpectralAngleMapper, "image")
_SpectralDistortionIndex = deprecated_class(SpectralDistortionIndex, "image")
_StructuralSimilarityIndexMeasure = deprecated_class(StructuralSimilarityIndexMeasure, "image")
_TotalVariation = deprecated_class(TotalVariation, "image")
_UniversalImageQualityIndex = deprecated_class(UniversalImageQualityIndex, "image")
