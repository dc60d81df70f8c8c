"""Image metrics (API parity: reference ``image/__init__.py``)."""
from torchmetrics_forked_amd.image.generative import (
    FrechetInceptionDistance,
    InceptionScore,
    KernelInceptionDistance,
    LearnedPerceptualImagePatchSimilarity,
    MemorizationInformedFrechetInceptionDistance,
    PerceptualPathLength,
)
from torchmetrics_forked_amd.image._simple import (
    ErrorRelativeGlobalDimensionlessSynthesis,
    MultiScaleStructuralSimilarityIndexMeasure,
    PeakSignalNoiseRatio,
    PeakSignalNoiseRatioWithBlockedEffect,
    RelativeAverageSpectralError,
    RootMeanSquaredErrorUsingSlidingWindow,
    SpectralAngleMapper,
    SpectralDistortionIndex,
    StructuralSimilarityIndexMeasure,
    TotalVariation,
    UniversalImageQualityIndex,
    VisualInformationFidelity,
)

__all__ = [
    "FrechetInceptionDistance", "InceptionScore", "KernelInceptionDistance", "LearnedPerceptualImagePatchSimilarity",
    "MemorizationInformedFrechetInceptionDistance", "PerceptualPathLength",
    "ErrorRelativeGlobalDimensionlessSynthesis", "MultiScaleStructuralSimilarityIndexMeasure", "PeakSignalNoiseRatio",
    "PeakSignalNoiseRatioWithBlockedEffect", "RelativeAverageSpectralError", "RootMeanSquaredErrorUsingSlidingWindow",
    "SpectralAngleMapper", "SpectralDistortionIndex", "StructuralSimilarityIndexMeasure", "TotalVariation",
    "UniversalImageQualityIndex", "VisualInformationFidelity",
]
