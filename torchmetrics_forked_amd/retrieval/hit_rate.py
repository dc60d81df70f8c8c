"""Module-path alias of reference ``src/torchmetrics/retrieval/hit_rate.py`` (the implementation lives in ``torchmetrics_forked_amd.retrieval``;
this file keeps ``from torchmetrics.retrieval.hit_rate import ...`` style imports working)."""
from torchmetrics_forked_amd.retrieval import RetrievalHitRate

__all__ = ['RetrievalHitRate']
