"""Module-path alias of reference ``src/torchmetrics/image/psnr.py`` (the implementation lives in ``torchmetrics_forked_amd.image``;
this file keeps ``from torchmetrics.image.psnr import ...`` style imports working)."""
from torchmetrics_forked_amd.image import PeakSignalNoiseRatio

__all__ = ['PeakSignalNoiseRatio']
