"""Module-path alias of reference ``src/torchmetrics/regression/kendall.py`` (the implementation lives in ``torchmetrics_forked_amd.regression``;
this file keeps ``from torchmetrics.regression.kendall import ...`` style imports working)."""
from torchmetrics_forked_amd.regression import KendallRankCorrCoef

__all__ = ['KendallRankCorrCoef']
