"""Re-export (reference ``detection/diou.py``)."""
from torchmetrics_forked_amd.detection.iou import DistanceIntersectionOverUnion

__all__ = ["DistanceIntersectionOverUnion"]
