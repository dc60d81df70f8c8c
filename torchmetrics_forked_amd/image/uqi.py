"""Module-path alias of reference ``src/torchmetrics/image/uqi.py`` (the implementation lives in ``torchmetrics_forked_amd.image``;
this file keeps ``from torchmetrics.image.uqi import ...`` style imports working)."""
from torchmetrics_forked_amd.image import UniversalImageQualityIndex

__all__ = ['UniversalImageQualityIndex']
