"""Intersection over union (API parity: reference ``functional/detection/iou.py``)."""
from typing import Optional

import torch

from torchmetrics_forked_amd.functional.detection._box_ops import pairwise_box_overlap


def _iou_update(
    preds: torch.Tensor, target: torch.Tensor, iou_threshold: Optional[float], replacement_val: float = 0
) -> torch.Tensor:
    iou = pairwise_box_overlap(preds, target, "iou")
    if iou_threshold is not None:
        iou = torch.where(iou < iou_threshold, torch.full_like(iou, replacement_val), iou)
    return iou


def _iou_compute(iou: torch.Tensor, aggregate: bool = True) -> torch.Tensor:
    if not aggregate:
        return iou
    return iou.diag().mean() if iou.numel() > 0 else torch.tensor(0.0, device=iou.device)


def intersection_over_union(
    preds: torch.Tensor,
    target: torch.Tensor,
    iou_threshold: Optional[float] = None,
    replacement_val: float = 0,
    aggregate: bool = True,
) -> torch.Tensor:
    return _iou_compute(_iou_update(preds, target, iou_threshold, replacement_val), aggregate)
