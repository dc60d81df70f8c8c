"""Module-path alias of reference ``src/torchmetrics/retrieval/r_precision.py`` (the implementation lives in ``torchmetrics_forked_amd.retrieval``;
this file keeps ``from torchmetrics.retrieval.r_precision import ...`` style imports working)."""
from torchmetrics_forked_amd.retrieval import RetrievalRPrecision

__all__ = ['RetrievalRPrecision']
