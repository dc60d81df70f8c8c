"""Module-path alias of reference ``src/torchmetrics/regression/log_cosh.py`` (the implementation lives in ``torchmetrics_forked_amd.regression``;
this file keeps ``from torchmetrics.regression.log_cosh import ...`` style imports working)."""
from torchmetrics_forked_amd.regression import LogCoshError

__all__ = ['LogCoshError']
