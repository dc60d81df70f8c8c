"""Re-export (reference ``detection/giou.py``)."""
from torchmetrics_forked_amd.detection.iou import GeneralizedIntersectionOverUnion

__all__ = ["GeneralizedIntersectionOverUnion"]
