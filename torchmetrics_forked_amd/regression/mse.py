"""Module-path alias of reference ``src/torchmetrics/regression/mse.py`` (the implementation lives in ``torchmetrics_forked_amd.regression``;
this file keeps ``from torchmetrics.regression.mse import ...`` style imports working)."""
from torchmetrics_forked_amd.regression import MeanSquaredError

__all__ = ['MeanSquaredError']
