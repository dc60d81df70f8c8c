"""Module-path alias of reference ``src/torchmetrics/retrieval/fall_out.py`` (the implementation lives in ``torchmetrics_forked_amd.retrieval``;
this file keeps ``from torchmetrics.retrieval.fall_out import ...`` style imports working)."""
from torchmetrics_forked_amd.retrieval import RetrievalFallOut

__all__ = ['RetrievalFallOut']
