"""Module-path alias of reference ``src/torchmetrics/regression/concordance.py`` (the implementation lives in ``torchmetrics_forked_amd.regression``;
this file keeps ``from torchmetrics.regression.concordance import ...`` style imports working)."""
from torchmetrics_forked_amd.regression import ConcordanceCorrCoef

__all__ = ['ConcordanceCorrCoef']
