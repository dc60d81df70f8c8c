"""Module-path alias of reference ``src/torchmetrics/image/kid.py`` (the implementation lives in ``torchmetrics_forked_amd.image``;
this file keeps ``from torchmetrics.image.kid import ...`` style imports working)."""
from torchmetrics_forked_amd.image.generative import maximum_mean_discrepancy, poly_kernel, poly_mmd, KernelInceptionDistance

__all__ = ['maximum_mean_discrepancy', 'poly_kernel', 'poly_mmd', 'KernelInceptionDistance']
