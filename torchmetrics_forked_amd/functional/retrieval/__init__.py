"""Functional retrieval metrics (API parity: reference ``functional/retrieval/__init__.py``); single-query forms of
the segmented engine in ``_grouped``."""
from torchmetrics_forked_amd.functional.retrieval.average_precision import retrieval_average_precision
from torchmetrics_forked_amd.functional.retrieval.fall_out import retrieval_fall_out
from torchmetrics_forked_amd.functional.retrieval.hit_rate import retrieval_hit_rate
from torchmetrics_forked_amd.functional.retrieval.ndcg import retrieval_normalized_dcg
from torchmetrics_forked_amd.functional.retrieval.precision import retrieval_precision
from torchmetrics_forked_amd.functional.retrieval.precision_recall_curve import retrieval_precision_recall_curve
from torchmetrics_forked_amd.functional.retrieval.r_precision import retrieval_r_precision
from torchmetrics_forked_amd.functional.retrieval.recall import retrieval_recall
from torchmetrics_forked_amd.functional.retrieval.reciprocal_rank import retrieval_reciprocal_rank

__all__ = [
    "retrieval_average_precision", "retrieval_fall_out", "retrieval_hit_rate", "retrieval_normalized_dcg",
    "retrieval_precision", "retrieval_precision_recall_curve", "retrieval_r_precision", "retrieval_recall",
    "retrieval_reciprocal_rank",
]
