"""Module-path alias of reference ``src/torchmetrics/clustering/rand_score.py`` (the implementation lives in ``torchmetrics_forked_amd.clustering``;
this file keeps ``from torchmetrics.clustering.rand_score import ...`` style imports working)."""
from torchmetrics_forked_amd.clustering import RandScore

__all__ = ['RandScore']
