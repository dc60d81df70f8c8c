"""Retrieval metrics (API parity: reference ``retrieval/__init__.py``)."""
from torchmetrics_forked_amd.retrieval.base import RetrievalMetric
from torchmetrics_forked_amd.retrieval.metrics import (
    RetrievalFallOut,
    RetrievalHitRate,
    RetrievalMAP,
    RetrievalMRR,
    RetrievalNormalizedDCG,
    RetrievalPrecision,
    RetrievalRecall,
    RetrievalRPrecision,
)
from torchmetrics_forked_amd.retrieval.precision_recall_curve import (
    RetrievalPrecisionRecallCurve,
    RetrievalRecallAtFixedPrecision,
)

__all__ = [
    "RetrievalFallOut", "RetrievalHitRate", "RetrievalMAP", "RetrievalMetric", "RetrievalMRR", "RetrievalNormalizedDCG",
    "RetrievalPrecision", "RetrievalPrecisionRecallCurve", "RetrievalRecall", "RetrievalRecallAtFixedPrecision",
    "RetrievalRPrecision",
]
