"""Functional pairwise similarities / distances (API parity: reference ``functional/pairwise/__init__.py``)."""
from torchmetrics_forked_amd.functional.pairwise.cosine import pairwise_cosine_similarity
from torchmetrics_forked_amd.functional.pairwise.euclidean import pairwise_euclidean_distance
from torchmetrics_forked_amd.functional.pairwise.linear import pairwise_linear_similarity
from torchmetrics_forked_amd.functional.pairwise.manhattan import pairwise_manhattan_distance
from torchmetrics_forked_amd.functional.pairwise.minkowski import pairwise_minkowski_distance

__all__ = [
    "pairwise_cosine_similarity", "pairwise_euclidean_distance", "pairwise_linear_similarity",
    "pairwise_manhattan_distance", "pairwise_minkowski_distance",
]
