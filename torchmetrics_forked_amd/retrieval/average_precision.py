"""Module-path alias of reference ``src/torchmetrics/retrieval/average_precision.py`` (the implementation lives in ``torchmetrics_forked_amd.retrieval``;
this file keeps ``from torchmetrics.retrieval.average_precision import ...`` style imports working)."""
from torchmetrics_forked_amd.retrieval import RetrievalMAP

__all__ = ['RetrievalMAP']
