"""Module-path alias of reference ``src/torchmetrics/image/lpip.py`` (the implementation lives in ``torchmetrics_forked_amd.image``;
this file keeps ``from torchmetrics.image.lpip import ...`` style imports working)."""
from torchmetrics_forked_amd.image import LearnedPerceptualImagePatchSimilarity

__all__ = ['LearnedPerceptualImagePatchSimilarity']
