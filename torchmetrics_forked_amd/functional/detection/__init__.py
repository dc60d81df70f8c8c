"""Functional detection metrics (reference ``functional/detection/__init__.py``)."""
from torchmetrics_forked_amd.functional.detection.ciou import complete_intersection_over_union
from torchmetrics_forked_amd.functional.detection.diou import distance_intersection_over_union
from torchmetrics_forked_amd.functional.detection.giou import generalized_intersection_over_union
from torchmetrics_forked_amd.functional.detection.iou import intersection_over_union
from torchmetrics_forked_amd.functional.detection.panoptic_qualities import modified_panoptic_quality, panoptic_quality

__all__ = [
    "complete_intersection_over_union",
    "distance_intersection_over_union",
    "generalized_intersection_over_union",
    "intersection_over_union",
    "modified_panoptic_quality",
    "panoptic_quality",
]
