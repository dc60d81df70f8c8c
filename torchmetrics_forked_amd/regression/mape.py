"""Module-path alias of reference ``src/torchmetrics/regression/mape.py`` (the implementation lives in ``torchmetrics_forked_amd.regression``;
this file keeps ``from torchmetrics.regression.mape import ...`` style imports working)."""
from torchmetrics_forked_amd.regression import MeanAbsolutePercentageError

__all__ = ['MeanAbsolutePercentageError']
