"""Module-path alias of reference ``src/torchmetrics/regression/spearman.py`` (the implementation lives in ``torchmetrics_forked_amd.regression``;
this file keeps ``from torchmetrics.regression.spearman import ...`` style imports working)."""
from torchmetrics_forked_amd.regression import SpearmanCorrCoef

__all__ = ['SpearmanCorrCoef']
