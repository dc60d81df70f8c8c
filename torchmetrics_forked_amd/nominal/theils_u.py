"""Module-path alias of reference ``src/torchmetrics/nominal/theils_u.py`` (the implementation lives in ``torchmetrics_forked_amd.nominal``;
this file keeps ``from torchmetrics.nominal.theils_u import ...`` style imports working)."""
from torchmetrics_forked_amd.nominal import TheilsU

__all__ = ['TheilsU']
