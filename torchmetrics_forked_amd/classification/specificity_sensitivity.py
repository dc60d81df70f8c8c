"""Specificity at sensitivity modules (reference ``classification/specificity_sensitivity.py``); see ``_fixed_point``."""
from torchmetrics_forked_amd.classification._fixed_point import (  # noqa: F401
    BinarySpecificityAtSensitivity,
    MulticlassSpecificityAtSensitivity,
    MultilabelSpecificityAtSensitivity,
    SpecificityAtSensitivity,
)
