"""Module-path alias of reference ``src/torchmetrics/regression/explained_variance.py`` (the implementation lives in ``torchmetrics_forked_amd.regression``;
this file keeps ``from torchmetrics.regression.explained_variance import ...`` style imports working)."""
from torchmetrics_forked_amd.regression import ExplainedVariance

__all__ = ['ExplainedVariance']
