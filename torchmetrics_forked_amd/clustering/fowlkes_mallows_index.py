"""Module-path alias of reference ``src/torchmetrics/clustering/fowlkes_mallows_index.py`` (the implementation lives in ``torchmetrics_forked_amd.clustering``;
this file keeps ``from torchmetrics.clustering.fowlkes_mallows_index import ...`` style imports working)."""
from torchmetrics_forked_amd.clustering import FowlkesMallowsIndex

__all__ = ['FowlkesMallowsIndex']
