"""Deprecated root-import shims for ``detection`` (reference ``detection/_deprecated.py``)."""
from torchmetrics_forked_amd.detection import (
    ModifiedPanopticQuality,
    PanopticQuality,
)
from torchmetrics_forked_amd.utilities.deprecation import deprecated_class

_ModifiedPanopticQuality = deprecated_class(ModifiedPanopticQuality, "detection")
_PanopticQuality = deprecated_class(PanopticQuality, "detection")
