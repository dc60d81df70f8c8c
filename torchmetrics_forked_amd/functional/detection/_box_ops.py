"""Box utilities (torchvision-equivalent semantics, implemented here; SURVEY §2.9: no torchvision dependency).

Pairwise overlap matrices use the tiled gfx950 kernel ``tmx::box_pairwise`` on GPU tensors without autograd,
and the eager PyTorch formulas otherwise."""
from typing import Tuple

import math

import torch
from torch import Tensor

from torchmetrics_forked_amd import ops

_MODES = {"iou": 0, "giou": 1, "diou": 2, "ciou": 3}


def box_convert(boxes: Tensor, in_fmt: str, out_fmt: str) -> Tensor:
    """Convert between ``xyxy``, ``xywh`` and ``cxcywh``."""
    if in_fmt == out_fmt:
        return boxes.clone()
    if in_fmt == "xywh":
        x, y, w, h = boxes.unbind(-1)
        xyxy = torch.stack([x, y, x + w, y + h], dim=-1)
    elif in_fmt == "cxcywh":
        cx, cy, w, h = boxes.unbind(-1)
        xyxy = torch.stack([cx - 0.5 * w, cy - 0.5 * h, cx + 0.5 * w, cy + 0.5 * h], dim=-1)
    elif in_fmt == "xyxy":
        xyxy = boxes
    else:
        raise ValueError(f"Unsupported box format {in_fmt}")
    if out_fmt == "xyxy":
        return xyxy
    if out_fmt == "xywh":  # (two kernels instead of unbind + two subtractions + stack; the same values)
        lo = xyxy[..., :2]
        return torch.cat([lo, xyxy[..., 2:] - lo], dim=-1)
    x0, y0, x1, y1 = xyxy.unbind(-1)
    if out_fmt == "cxcywh":
        return torch.stack([(x0 + x1) / 2, (y0 + y1) / 2, x1 - x0, y1 - y0], dim=-1)
    raise ValueError(f"Unsupported box format {out_fmt}")


def box_area(boxes: Tensor) -> Tensor:
    return (boxes[:, 2] - boxes[:, 0]) * (boxes[:, 3] - boxes[:, 1])


def _upcast(t: Tensor) -> Tensor:
    return t if t.is_floating_point() else t.float()


def _inter_union(b1: Tensor, b2: Tensor) -> Tuple[Tensor, Tensor]:
    area1, area2 = box_area(b1), box_area(b2)
    lt = torch.max(b1[:, None, :2], b2[:, :2])
    rb = torch.min(b1[:, None, 2:], b2[:, 2:])
    wh = _upcast(rb - lt).clamp(min=0)
    inter = wh[:, :, 0] * wh[:, :, 1]
    return inter, area1[:, None] + area2 - inter


def _eager(b1: Tensor, b2: Tensor, mode: str) -> Tensor:
    inter, union = _inter_union(b1, b2)
    iou = inter / union
    if mode == "iou":
        return iou
    lti = torch.min(b1[:, None, :2], b2[:, :2])
    rbi = torch.max(b1[:, None, 2:], b2[:, 2:])
    whi = _upcast(rbi - lti).clamp(min=0)
    if mode == "giou":
        areai = whi[:, :, 0] * whi[:, :, 1]
        return iou - (areai - union) / areai
    eps = 1e-7
    diag = whi[:, :, 0] ** 2 + whi[:, :, 1] ** 2 + eps
    xp, yp = (b1[:, 0] + b1[:, 2]) / 2, (b1[:, 1] + b1[:, 3]) / 2
    xg, yg = (b2[:, 0] + b2[:, 2]) / 2, (b2[:, 1] + b2[:, 3]) / 2
    cdist = _upcast(xp[:, None] - xg[None, :]) ** 2 + _upcast(yp[:, None] - yg[None, :]) ** 2
    diou = iou - cdist / diag
    if mode == "diou":
        return diou
    w_p, h_p = b1[:, None, 2] - b1[:, None, 0], b1[:, None, 3] - b1[:, None, 1]
    w_g, h_g = b2[:, 2] - b2[:, 0], b2[:, 3] - b2[:, 1]
    v = (4 / (math.pi**2)) * torch.pow(torch.atan(w_p / h_p) - torch.atan(w_g / h_g), 2)
    with torch.no_grad():
        alpha = v / (1 - iou + v + eps)
    return diou - alpha * v


def pairwise_box_overlap(b1: Tensor, b2: Tensor, mode: str = "iou") -> Tensor:
    if b1.numel() == 0:
        b1 = b1.reshape(0, 4)
    if b2.numel() == 0:
        b2 = b2.reshape(0, 4)
    grad = torch.is_grad_enabled() and (b1.requires_grad or b2.requires_grad)
    if b1.is_cuda and not grad and b1.dtype in (torch.float32, torch.float16, torch.bfloat16) and ops.use_native(b1):
        return torch.ops.tmx.box_pairwise(b1, b2, _MODES[mode]).to(b1.dtype)
    return _eager(b1, b2, mode)


def box_iou(b1: Tensor, b2: Tensor) -> Tensor:
    return pairwise_box_overlap(b1, b2, "iou")


def generalized_box_iou(b1: Tensor, b2: Tensor) -> Tensor:
    return pairwise_box_overlap(b1, b2, "giou")


def distance_box_iou(b1: Tensor, b2: Tensor) -> Tensor:
    return pairwise_box_overlap(b1, b2, "diou")


def complete_box_iou(b1: Tensor, b2: Tensor) -> Tensor:
    return pairwise_box_overlap(b1, b2, "ciou")
