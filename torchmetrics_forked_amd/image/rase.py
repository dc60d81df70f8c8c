"""Module-path alias of reference ``src/torchmetrics/image/rase.py`` (the implementation lives in ``torchmetrics_forked_amd.image``;
this file keeps ``from torchmetrics.image.rase import ...`` style imports working)."""
from torchmetrics_forked_amd.image import RelativeAverageSpectralError

__all__ = ['RelativeAverageSpectralError']
