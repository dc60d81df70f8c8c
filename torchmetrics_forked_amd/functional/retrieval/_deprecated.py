"""Deprecated ``functional`` root-import shims for ``retrieval`` (reference ``functional/retrieval/_deprecated.py``)."""
from torchmetrics_forked_amd.functional.retrieval import (
    retrieval_average_precision,
    retrieval_fall_out,
    retrieval_hit_rate,
    retrieval_normalized_dcg,
    retrieval_precision,
    retrieval_precision_recall_curve,
    retrieval_r_precision,
    retrieval_recall,
    retrieval_reciprocal_rank,
)
from torchmetrics_forked_amd.utilities.deprecation import deprecated_func

_retrieval_average_precision = deprecated_func(retrieval_average_precision, "retrieval")
_retrieval_fall_out = deprecated_func(retrieval_fall_out, "retrieval")
_retrieval_hit_rate = deprecated_func(retrieval_hit_rate, "retrieval")
_retrieval_normalized_dcg = deprecated_func(retrieval_normalized_dcg, "retrieval")
_retrieval_precision = deprecated_func(retrieval_precision, "retrieval")
_retrieval_precision_recall_curve = deprecated_func(retrieval_precision_recall_curve, "retrieval")
_retrieval_r_precision = deprecated_func(retrieval_r_precision, "retrieval")
_retrieval_recall = deprecated_func(retrieval_recall, "retrieval")
_retrieval_reciprocal_rank = deprecated_func(retrieval_reciprocal_rank, "retrieval")
