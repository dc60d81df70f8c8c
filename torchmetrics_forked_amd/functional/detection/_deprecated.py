"""Deprecated ``functional`` root-import shims for ``detection`` (reference ``functional/detection/_deprecated.py``)."""
from torchmetrics_forked_amd.functional.detection import (
    panoptic_quality,
)
from torchmetrics_forked_amd.utilities.deprecation import deprecated_func

_panoptic_quality = deprecated_func(panoptic_quality, "detection")
