"""Module-path alias of reference ``src/torchmetrics/nominal/tschuprows.py`` (the implementation lives in ``torchmetrics_forked_amd.nominal``;
this file keeps ``from torchmetrics.nominal.tschuprows import ...`` style imports working)."""
from torchmetrics_forked_amd.nominal import TschuprowsT

__all__ = ['TschuprowsT']
