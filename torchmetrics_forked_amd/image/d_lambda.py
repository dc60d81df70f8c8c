"""Module-path alias of reference ``src/torchmetrics/image/d_lambda.py`` (the implementation lives in ``torchmetrics_forked_amd.image``;
this file keeps ``from torchmetrics.image.d_lambda import ...`` style imports working)."""
from torchmetrics_forked_amd.image import SpectralDistortionIndex

__all__ = ['SpectralDistortionIndex']
