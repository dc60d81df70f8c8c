"""Module-path alias of reference ``src/torchmetrics/clustering/davies_bouldin_score.py`` (the implementation lives in ``torchmetrics_forked_amd.clustering``;
this file keeps ``from torchmetrics.clustering.davies_bouldin_score import ...`` style imports working)."""
from torchmetrics_forked_amd.clustering import DaviesBouldinScore

__all__ = ['DaviesBouldinScore']
