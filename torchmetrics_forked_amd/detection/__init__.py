"""Detection metrics (reference ``detection/__init__.py``): mAP/mAR, IoU family, panoptic quality."""
from torchmetrics_forked_amd.detection.iou import (
    CompleteIntersectionOverUnion,
    DistanceIntersectionOverUnion,
    GeneralizedIntersectionOverUnion,
    IntersectionOverUnion,
)
from torchmetrics_forked_amd.detection.mean_ap import MeanAveragePrecision
from torchmetrics_forked_amd.detection.panoptic_qualities import ModifiedPanopticQuality, PanopticQuality

__all__ = [
    "CompleteIntersectionOverUnion",
    "DistanceIntersectionOverUnion",
    "GeneralizedIntersectionOverUnion",
    "IntersectionOverUnion",
    "MeanAveragePrecision",
    "ModifiedPanopticQuality",
    "PanopticQuality",
]
