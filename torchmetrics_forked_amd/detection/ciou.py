"""Re-export (reference ``detection/ciou.py``)."""
from torchmetrics_forked_amd.detection.iou import CompleteIntersectionOverUnion

__all__ = ["CompleteIntersectionOverUnion"]
