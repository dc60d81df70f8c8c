"""Module-path alias of reference ``src/torchmetrics/regression/symmetric_mape.py`` (the implementation lives in ``torchmetrics_forked_amd.regression``;
this file keeps ``from torchmetrics.regression.symmetric_mape import ...`` style imports working)."""
from torchmetrics_forked_amd.regression import SymmetricMeanAbsolutePercentageError

__all__ = ['SymmetricMeanAbsolutePercentageError']
