"""MI355X-native metrics framework (capabilities of TorchMetrics 1.3; gfx950 HIP kernels + RCCL sync)."""
import logging as __logging

from torchmetrics_forked_amd.__about__ import __version__  # noqa: F401

_logger = __logging.getLogger("torchmetrics_forked_amd")
_logger.addHandler(__logging.StreamHandler())
_logger.setLevel(__logging.INFO)

from torchmetrics_forked_amd import functional  # noqa: E402
from torchmetrics_forked_amd import (  # noqa: E402,F401
    audio,
    clustering,
    detection,
    image,
    models,
    multimodal,
    nominal,
    regression,
    retrieval,
    text,
    utilities,
    wrappers,
)
from torchmetrics_forked_amd.aggregation import (  # noqa: E402
    CatMetric,
    MaxMetric,
    MeanMetric,
    MinMetric,
    RunningMean,
    RunningSum,
    SumMetric,
)
from torchmetrics_forked_amd.classification import *  # noqa: E402,F401,F403
from torchmetrics_forked_amd.collections import MetricCollection  # noqa: E402
from torchmetrics_forked_amd.metric import CompositionalMetric, Metric  # noqa: E402
from torchmetrics_forked_amd.nominal import *  # noqa: E402,F401,F403
from torchmetrics_forked_amd.regression import *  # noqa: E402,F401,F403
from torchmetrics_forked_amd.wrappers import (  # noqa: E402
    BootStrapper,
    ClasswiseWrapper,
    MetricTracker,
    MinMaxMetric,
    MultioutputWrapper,
    MultitaskWrapper,
)

# domain metrics importable from the root with a FutureWarning (reference ``__init__.py:67-140``)
from torchmetrics_forked_amd.audio._deprecated import _PermutationInvariantTraining as PermutationInvariantTraining  # noqa: E402
from torchmetrics_forked_amd.audio._deprecated import _ScaleInvariantSignalDistortionRatio as ScaleInvariantSignalDistortionRatio  # noqa: E402
from torchmetrics_forked_amd.audio._deprecated import _ScaleInvariantSignalNoiseRatio as ScaleInvariantSignalNoiseRatio  # noqa: E402
from torchmetrics_forked_amd.audio._deprecated import _SignalDistortionRatio as SignalDistortionRatio  # noqa: E402
from torchmetrics_forked_amd.audio._deprecated import _SignalNoiseRatio as SignalNoiseRatio  # noqa: E402
from torchmetrics_forked_amd.detection._deprecated import _ModifiedPanopticQuality as ModifiedPanopticQuality  # noqa: E402
from torchmetrics_forked_amd.detection._deprecated import _PanopticQuality as PanopticQuality  # noqa: E402
from torchmetrics_forked_amd.image._deprecated import _ErrorRelativeGlobalDimensionlessSynthesis as ErrorRelativeGlobalDimensionlessSynthesis  # noqa: E402
from torchmetrics_forked_amd.image._deprecated import _MultiScaleStructuralSimilarityIndexMeasure as MultiScaleStructuralSimilarityIndexMeasure  # noqa: E402
from torchmetrics_forked_amd.image._deprecated import _PeakSignalNoiseRatio as PeakSignalNoiseRatio  # noqa: E402
from torchmetrics_forked_amd.image._deprecated import _RelativeAverageSpectralError as RelativeAverageSpectralError  # noqa: E402
from torchmetrics_forked_amd.image._deprecated import _RootMeanSquaredErrorUsingSlidingWindow as RootMeanSquaredErrorUsingSlidingWindow  # noqa: E402
from torchmetrics_forked_amd.image._deprecated import _SpectralAngleMapper as SpectralAngleMapper  # noqa: E402
from torchmetrics_forked_amd.image._deprecated import _SpectralDistortionIndex as SpectralDistortionIndex  # noqa: E402
from torchmetrics_forked_amd.image._deprecated import _StructuralSimilarityIndexMeasure as StructuralSimilarityIndexMeasure  # noqa: E402
from torchmetrics_forked_amd.image._deprecated import _TotalVariation as TotalVariation  # noqa: E402
from torchmetrics_forked_amd.image._deprecated import _UniversalImageQualityIndex as UniversalImageQualityIndex  # noqa: E402
from torchmetrics_forked_amd.retrieval._deprecated import _RetrievalFallOut as RetrievalFallOut  # noqa: E402
from torchmetrics_forked_amd.retrieval._deprecated import _RetrievalHitRate as RetrievalHitRate  # noqa: E402
from torchmetrics_forked_amd.retrieval._deprecated import _RetrievalMAP as RetrievalMAP  # noqa: E402
from torchmetrics_forked_amd.retrieval._deprecated import _RetrievalMRR as RetrievalMRR  # noqa: E402
from torchmetrics_forked_amd.retrieval._deprecated import _RetrievalNormalizedDCG as RetrievalNormalizedDCG  # noqa: E402
from torchmetrics_forked_amd.retrieval._deprecated import _RetrievalPrecision as RetrievalPrecision  # noqa: E402
from torchmetrics_forked_amd.retrieval._deprecated import _RetrievalPrecisionRecallCurve as RetrievalPrecisionRecallCurve  # noqa: E402
from torchmetrics_forked_amd.retrieval._deprecated import _RetrievalRecall as RetrievalRecall  # noqa: E402
from torchmetrics_forked_amd.retrieval._deprecated import _RetrievalRecallAtFixedPrecision as RetrievalRecallAtFixedPrecision  # noqa: E402
from torchmetrics_forked_amd.retrieval._deprecated import _RetrievalRPrecision as RetrievalRPrecision  # noqa: E402
from torchmetrics_forked_amd.text._deprecated import _BLEUScore as BLEUScore  # noqa: E402
from torchmetrics_forked_amd.text._deprecated import _CharErrorRate as CharErrorRate  # noqa: E402
from torchmetrics_forked_amd.text._deprecated import _CHRFScore as CHRFScore  # noqa: E402
from torchmetrics_forked_amd.text._deprecated import _ExtendedEditDistance as ExtendedEditDistance  # noqa: E402
from torchmetrics_forked_amd.text._deprecated import _MatchErrorRate as MatchErrorRate  # noqa: E402
from torchmetrics_forked_amd.text._deprecated import _Perplexity as Perplexity  # noqa: E402
from torchmetrics_forked_amd.text._deprecated import _SacreBLEUScore as SacreBLEUScore  # noqa: E402
from torchmetrics_forked_amd.text._deprecated import _SQuAD as SQuAD  # noqa: E402
from torchmetrics_forked_amd.text._deprecated import _TranslationEditRate as TranslationEditRate  # noqa: E402
from torchmetrics_forked_amd.text._deprecated import _WordErrorRate as WordErrorRate  # noqa: E402
from torchmetrics_forked_amd.text._deprecated import _WordInfoLost as WordInfoLost  # noqa: E402
from torchmetrics_forked_amd.text._deprecated import _WordInfoPreserved as WordInfoPreserved  # noqa: E402
