"""Module-path alias of reference ``src/torchmetrics/nominal/fleiss_kappa.py`` (the implementation lives in ``torchmetrics_forked_amd.nominal``;
this file keeps ``from torchmetrics.nominal.fleiss_kappa import ...`` style imports working)."""
from torchmetrics_forked_amd.nominal import FleissKappa

__all__ = ['FleissKappa']
