"""Module-path alias of reference ``src/torchmetrics/regression/wmape.py`` (the implementation lives in ``torchmetrics_forked_amd.regression``;
this file keeps ``from torchmetrics.regression.wmape import ...`` style imports working)."""
from torchmetrics_forked_amd.regression import WeightedMeanAbsolutePercentageError

__all__ = ['WeightedMeanAbsolutePercentageError']
