"""Recall at fixed precision modules (reference ``classification/recall_fixed_precision.py``); see ``_fixed_point``."""
from torchmetrics_forked_amd.classification._fixed_point import (  # noqa: F401
    BinaryRecallAtFixedPrecision,
    MulticlassRecallAtFixedPrecision,
    MultilabelRecallAtFixedPrecision,
    RecallAtFixedPrecision,
)
