"""Module-path alias of reference ``src/torchmetrics/regression/tweedie_deviance.py`` (the implementation lives in ``torchmetrics_forked_amd.regression``;
this file keeps ``from torchmetrics.regression.tweedie_deviance import ...`` style imports working)."""
from torchmetrics_forked_amd.regression import TweedieDevianceScore

__all__ = ['TweedieDevianceScore']
