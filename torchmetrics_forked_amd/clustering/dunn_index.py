"""Module-path alias of reference ``src/torchmetrics/clustering/dunn_index.py`` (the implementation lives in ``torchmetrics_forked_amd.clustering``;
this file keeps ``from torchmetrics.clustering.dunn_index import ...`` style imports working)."""
from torchmetrics_forked_amd.clustering import DunnIndex

__all__ = ['DunnIndex']
