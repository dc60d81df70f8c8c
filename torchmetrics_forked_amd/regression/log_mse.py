"""Module-path alias of reference ``src/torchmetrics/regression/log_mse.py`` (the implementation lives in ``torchmetrics_forked_amd.regression``;
this file keeps ``from torchmetrics.regression.log_mse import ...`` style imports working)."""
from torchmetrics_forked_amd.regression import MeanSquaredLogError

__all__ = ['MeanSquaredLogError']
