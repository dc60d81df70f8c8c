"""Module-path alias of reference ``src/torchmetrics/regression/pearson.py`` (the implementation lives in ``torchmetrics_forked_amd.regression``;
this file keeps ``from torchmetrics.regression.pearson import ...`` style imports working)."""
from torchmetrics_forked_amd.regression import PearsonCorrCoef

__all__ = ['PearsonCorrCoef']
