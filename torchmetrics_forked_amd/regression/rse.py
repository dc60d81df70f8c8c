"""Module-path alias of reference ``src/torchmetrics/regression/rse.py`` (the implementation lives in ``torchmetrics_forked_amd.regression``;
this file keeps ``from torchmetrics.regression.rse import ...`` style imports working)."""
from torchmetrics_forked_amd.regression import RelativeSquaredError

__all__ = ['RelativeSquaredError']
