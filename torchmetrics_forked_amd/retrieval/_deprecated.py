"""Deprecated root-import shims for ``retrieval`` (reference ``retrieval/_deprecated.py``)."""
from torchmetrics_forked_amd.retrieval import (
    RetrievalFallOut,
    RetrievalHitRate,
    RetrievalMAP,
    RetrievalMRR,
    RetrievalNormalizedDCG,
    RetrievalPrecision,
    RetrievalPrecisionRecallCurve,
    RetrievalRecall,
    RetrievalRecallAtFixedPrecision,
    RetrievalRPrecision,
)
from torchmetrics_forked_amd.utilities.deprecation import deprecated_class

_RetrievalFallOut = deprecated_class(RetrievalFallOut, "retrieval")
_RetrievalHitRate = deprecated_class(RetrievalHitRate, "retrieval")
_RetrievalMAP = deprecated_class(RetrievalMAP, "retrieval")
_RetrievalMRR = deprecated_class(RetrievalMRR, "retrieval")
_RetrievalNormalizedDCG = deprecated_class(RetrievalNormalizedDCG, "retrieval")
_RetrievalPrecision = deprecated_class(RetrievalPrecision, "retrieval")
_RetrievalPrecisionRecallCurve = deprecated_class(RetrievalPrecisionRecallCurve, "retrieval")
_RetrievalRecall = deprecated_class(RetrievalRecall, "retrieval")
_RetrievalRecallAtFixedPrecision = deprecated_class(RetrievalRecallAtFixedPrecision, "retrieval")
_RetrievalRPrecision = deprecated_class(RetrievalRPrecision, "retrieval")
