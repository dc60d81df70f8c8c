"""Module-path alias of reference ``src/torchmetrics/image/psnrb.py`` (the implementation lives in ``torchmetrics_forked_amd.image``;
this file keeps ``from torchmetrics.image.psnrb import ...`` style imports working)."""
from torchmetrics_forked_amd.image import PeakSignalNoiseRatioWithBlockedEffect

__all__ = ['PeakSignalNoiseRatioWithBlockedEffect']
