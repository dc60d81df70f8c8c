"""Module-path alias of reference ``src/torchmetrics/regression/cosine_similarity.py`` (the implementation lives in ``torchmetrics_forked_amd.regression``;
this file keeps ``from torchmetrics.regression.cosine_similarity import ...`` style imports working)."""
from torchmetrics_forked_amd.regression import CosineSimilarity

__all__ = ['CosineSimilarity']
