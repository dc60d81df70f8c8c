"""Module-path alias of reference ``src/torchmetrics/regression/minkowski.py`` (the implementation lives in ``torchmetrics_forked_amd.regression``;
this file keeps ``from torchmetrics.regression.minkowski import ...`` style imports working)."""
from torchmetrics_forked_amd.regression import MinkowskiDistance

__all__ = ['MinkowskiDistance']
