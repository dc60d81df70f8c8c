"""Module-path alias of reference ``src/torchmetrics/nominal/pearson.py`` (the implementation lives in ``torchmetrics_forked_amd.nominal``;
this file keeps ``from torchmetrics.nominal.pearson import ...`` style imports working)."""
from torchmetrics_forked_amd.nominal import PearsonsContingencyCoefficient

__all__ = ['PearsonsContingencyCoefficient']
