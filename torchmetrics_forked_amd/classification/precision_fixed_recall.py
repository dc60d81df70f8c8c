"""Precision at fixed recall modules (reference ``classification/precision_fixed_recall.py``); see ``_fixed_point``."""
from torchmetrics_forked_amd.classification._fixed_point import (  # noqa: F401
    BinaryPrecisionAtFixedRecall,
    MulticlassPrecisionAtFixedRecall,
    MultilabelPrecisionAtFixedRecall,
    PrecisionAtFixedRecall,
)
