"""Module-path alias of reference ``src/torchmetrics/image/ergas.py`` (the implementation lives in ``torchmetrics_forked_amd.image``;
this file keeps ``from torchmetrics.image.ergas import ...`` style imports working)."""
from torchmetrics_forked_amd.image import ErrorRelativeGlobalDimensionlessSynthesis

__all__ = ['ErrorRelativeGlobalDimensionlessSynthesis']
