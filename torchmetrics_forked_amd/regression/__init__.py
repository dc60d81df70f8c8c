"""Regression metrics (API parity: reference ``regression/__init__.py``)."""
from torchmetrics_forked_amd.regression.errors import (
    LogCoshError,
    MeanAbsoluteError,
    MeanAbsolutePercentageError,
    MeanSquaredError,
    MeanSquaredLogError,
    MinkowskiDistance,
    SymmetricMeanAbsolutePercentageError,
    TweedieDevianceScore,
    WeightedMeanAbsolutePercentageError,
)
from torchmetrics_forked_amd.regression.moments import (
    ConcordanceCorrCoef,
    ExplainedVariance,
    PearsonCorrCoef,
    R2Score,
    RelativeSquaredError,
)
from torchmetrics_forked_amd.regression.rank import CosineSimilarity, KendallRankCorrCoef, KLDivergence, SpearmanCorrCoef

__all__ = [
    "ConcordanceCorrCoef", "CosineSimilarity", "ExplainedVariance", "KendallRankCorrCoef", "KLDivergence",
    "LogCoshError", "MeanAbsoluteError", "MeanAbsolutePercentageError", "MeanSquaredError", "MeanSquaredLogError",
    "MinkowskiDistance", "PearsonCorrCoef", "R2Score", "RelativeSquaredError", "SpearmanCorrCoef",
    "SymmetricMeanAbsolutePercentageError", "TweedieDevianceScore", "WeightedMeanAbsolutePercentageError",
]
