"""Module-path alias of reference ``src/torchmetrics/image/perceptual_path_length.py`` (the implementation lives in ``torchmetrics_forked_amd.image``;
this file keeps ``from torchmetrics.image.perceptual_path_length import ...`` style imports working)."""
from torchmetrics_forked_amd.image import PerceptualPathLength

__all__ = ['PerceptualPathLength']
