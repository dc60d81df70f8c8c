"""Module-path alias of reference ``src/torchmetrics/retrieval/precision.py`` (the implementation lives in ``torchmetrics_forked_amd.retrieval``;
this file keeps ``from torchmetrics.retrieval.precision import ...`` style imports working)."""
from torchmetrics_forked_amd.retrieval import RetrievalPrecision

__all__ = ['RetrievalPrecision']
