"""Module-path alias of reference ``src/torchmetrics/retrieval/reciprocal_rank.py`` (the implementation lives in ``torchmetrics_forked_amd.retrieval``;
this file keeps ``from torchmetrics.retrieval.reciprocal_rank import ...`` style imports working)."""
from torchmetrics_forked_amd.retrieval import RetrievalMRR

__all__ = ['RetrievalMRR']
