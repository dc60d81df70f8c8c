"""Module-path alias of reference ``src/torchmetrics/regression/mae.py`` (the implementation lives in ``torchmetrics_forked_amd.regression``;
this file keeps ``from torchmetrics.regression.mae import ...`` style imports working)."""
from torchmetrics_forked_amd.regression import MeanAbsoluteError

__all__ = ['MeanAbsoluteError']
