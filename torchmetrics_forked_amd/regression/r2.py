"""Module-path alias of reference ``src/torchmetrics/regression/r2.py`` (the implementation lives in ``torchmetrics_forked_amd.regression``;
this file keeps ``from torchmetrics.regression.r2 import ...`` style imports working)."""
from torchmetrics_forked_amd.regression import R2Score

__all__ = ['R2Score']
