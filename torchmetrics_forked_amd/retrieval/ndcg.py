"""Module-path alias of reference ``src/torchmetrics/retrieval/ndcg.py`` (the implementation lives in ``torchmetrics_forked_amd.retrieval``;
this file keeps ``from torchmetrics.retrieval.ndcg import ...`` style imports working)."""
from torchmetrics_forked_amd.retrieval import RetrievalNormalizedDCG

__all__ = ['RetrievalNormalizedDCG']
