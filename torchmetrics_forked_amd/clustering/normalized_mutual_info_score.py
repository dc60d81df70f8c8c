"""Module-path alias of reference ``src/torchmetrics/clustering/normalized_mutual_info_score.py`` (the implementation lives in ``torchmetrics_forked_amd.clustering``;
this file keeps ``from torchmetrics.clustering.normalized_mutual_info_score import ...`` style imports working)."""
from torchmetrics_forked_amd.clustering import NormalizedMutualInfoScore

__all__ = ['NormalizedMutualInfoScore']
