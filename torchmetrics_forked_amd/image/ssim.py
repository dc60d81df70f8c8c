"""Module-path alias of reference ``src/torchmetrics/image/ssim.py`` (the implementation lives in ``torchmetrics_forked_amd.image``;
this file keeps ``from torchmetrics.image.ssim import ...`` style imports working)."""
from torchmetrics_forked_amd.image import StructuralSimilarityIndexMeasure, MultiScaleStructuralSimilarityIndexMeasure

__all__ = ['StructuralSimilarityIndexMeasure', 'MultiScaleStructuralSimilarityIndexMeasure']
