"""Module-path alias of reference ``src/torchmetrics/image/inception.py`` (the implementation lives in ``torchmetrics_forked_amd.image``;
this file keeps ``from torchmetrics.image.inception import ...`` style imports working)."""
from torchmetrics_forked_amd.image import InceptionScore

__all__ = ['InceptionScore']
