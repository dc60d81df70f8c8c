"""Module-path alias of reference ``src/torchmetrics/image/vif.py`` (the implementation lives in ``torchmetrics_forked_amd.image``;
this file keeps ``from torchmetrics.image.vif import ...`` style imports working)."""
from torchmetrics_forked_amd.image import VisualInformationFidelity

__all__ = ['VisualInformationFidelity']
