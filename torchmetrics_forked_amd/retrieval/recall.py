"""Module-path alias of reference ``src/torchmetrics/retrieval/recall.py`` (the implementation lives in ``torchmetrics_forked_amd.retrieval``;
this file keeps ``from torchmetrics.retrieval.recall import ...`` style imports working)."""
from torchmetrics_forked_amd.retrieval import RetrievalRecall

__all__ = ['RetrievalRecall']
