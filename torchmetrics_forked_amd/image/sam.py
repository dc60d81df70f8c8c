"""Module-path alias of reference ``src/torchmetrics/image/sam.py`` (the implementation lives in ``torchmetrics_forked_amd.image``;
this file keeps ``from torchmetrics.image.sam import ...`` style imports working)."""
from torchmetrics_forked_amd.image import SpectralAngleMapper

__all__ = ['SpectralAngleMapper']
