"""Module-path alias of reference ``src/torchmetrics/image/tv.py`` (the implementation lives in ``torchmetrics_forked_amd.image``;
this file keeps ``from torchmetrics.image.tv import ...`` style imports working)."""
from torchmetrics_forked_amd.image import TotalVariation

__all__ = ['TotalVariation']
