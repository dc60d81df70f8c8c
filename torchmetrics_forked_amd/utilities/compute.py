"""Numerically safe helpers (parity: reference ``utilities/compute.py:20-157``)."""
from typing import Optional, Tuple

import torch
from torch import Tensor

from torchmetrics_forked_amd.ops.sort import argsort as _argsort, sort as _sort


def _safe_matmul(x: Tensor, y: Tensor) -> Tensor:
    """``x @ y.T`` with fp16 promoted to fp32 on CPU (no half GEMM on CPU)."""
    if x.dtype == torch.float16 or y.dtype == torch.float16:
        return (x.float() @ y.T.float()).half()
    return x @ y.T


def _safe_xlogy(x: Tensor, y: Tensor) -> Tensor:
    """``x * log(y)`` with ``0 * log(0) = 0``."""
    res = x * torch.log(y)
    return torch.where(x == 0, torch.zeros_like(res), res)


def _safe_divide(num: Tensor, denom: Tensor) -> Tensor:
    """Division where ``denom == 0`` is treated as 1. Integer inputs are promoted to float.

    NOTE: like the reference (``utilities/compute.py:46-55``) ``denom`` is modified in place.
    """
    denom.masked_fill_(denom == 0.0, 1)  # in place, as the reference's boolean-index assignment (one kernel)
    num = num if num.is_floating_point() else num.float()
    denom = denom if denom.is_floating_point() else denom.float()
    return num / denom


def _adjust_weights_safe_divide(
    score: Tensor, average: Optional[str], multilabel: bool, tp: Tensor, fp: Tensor, fn: Tensor
) -> Tensor:
    """Macro / weighted averaging of a per-class score; macro drops classes with no tp/fp/fn (multiclass)."""
    if average is None or average == "none":
        return score
    if average == "weighted":
        weights = tp + fn
    else:
        weights = torch.ones_like(score)
        if not multilabel:
            weights.masked_fill_(tp + fp + fn == 0, 0.0)
    return _safe_divide(weights * score, weights.sum(-1, keepdim=True)).sum(-1)


def _auc_format_inputs(x: Tensor, y: Tensor) -> Tuple[Tensor, Tensor]:
    x = x.squeeze() if x.ndim > 1 else x
    y = y.squeeze() if y.ndim > 1 else y
    if x.ndim > 1 or y.ndim > 1:
        raise ValueError(
            f"Expected both `x` and `y` tensor to be 1d, but got tensors with dimension {x.ndim} and {y.ndim}"
        )
    if x.numel() != y.numel():
        raise ValueError(
            f"Expected the same number of elements in `x` and `y` tensor but received {x.numel()} and {y.numel()}"
        )
    return x, y


def _auc_compute_without_check(x: Tensor, y: Tensor, direction: float, axis: int = -1) -> Tensor:
    """Trapezoidal area, assuming ``x`` monotone along ``axis``."""
    with torch.no_grad():
        return torch.trapz(y, x, dim=axis) * direction


def _auc_compute(x: Tensor, y: Tensor, reorder: bool = False) -> Tensor:
    with torch.no_grad():
        if reorder:
            x, order = _sort(x)
            y = y[order]
        dx = x[1:] - x[:-1]
        direction = 1.0
        if (dx < 0).any():
            if not (dx <= 0).all():
                raise ValueError(
                    "The `x` tensor is neither increasing or decreasing. Try setting the reorder argument to `True`."
                )
            direction = -1.0
        return _auc_compute_without_check(x, y, direction)


def auc(x: Tensor, y: Tensor, reorder: bool = False) -> Tensor:
    """Area under the curve ``y(x)`` by the trapezoidal rule."""
    x, y = _auc_format_inputs(x, y)
    return _auc_compute(x, y, reorder=reorder)


def interp(x: Tensor, xp: Tensor, fp: Tensor) -> Tensor:
    """Piecewise-linear interpolation of ``(xp, fp)`` at ``x`` (``xp`` increasing).

    Uses a binary search (``searchsorted``) instead of the reference's O(M*K) broadcast compare
    (reference ``utilities/compute.py:134-157``); extrapolates linearly from the end segments.
    """
    slope = _safe_divide(fp[1:] - fp[:-1], xp[1:] - xp[:-1])
    intercept = fp[:-1] - slope * xp[:-1]
    # segment index = #(xp <= x) - 1, which is order independent (identical to the reference even when
    # xp is not monotone, e.g. macro-averaged PR curves); counted with a sort + binary search.
    idx = torch.searchsorted(_sort(xp)[0].contiguous(), x.contiguous(), right=True) - 1
    idx = idx.clamp(0, slope.numel() - 1)
    return slope[idx] * x + intercept[idx]


def macro_interp_sum(x: Tensor, xps: "list", fps: "list") -> "Optional[Tensor]":
    """Sum over the curves ``(xps[c], fps[c])`` of ``interp(x, xps[c], fps[c])`` in one GPU launch
    (csrc/interp.hip); ``None`` when the inputs do not qualify (CPU, non-fp32), so the caller keeps its loop."""
    from torchmetrics_forked_amd import ops

    if not (x.is_cuda and x.dtype == torch.float32 and ops.use_native(x)):
        return None
    if any(t.dtype != torch.float32 or not t.is_cuda for t in list(xps) + list(fps)):
        return None
    lens = torch.tensor([0] + [t.numel() for t in xps], dtype=torch.long)
    off = torch.cumsum(lens, 0).to(x.device)
    xp = torch.cat([t.reshape(-1) for t in xps])
    fp = torch.cat([t.reshape(-1) for t in fps])
    cls = torch.repeat_interleave(torch.arange(len(xps), device=x.device), lens[1:].to(x.device))
    # every class's values sorted inside its segment: stable sort by value, then stable by class
    o1 = _argsort(xp)
    o2 = _argsort(cls[o1])
    xs = xp[o1[o2]]
    return torch.ops.tmx.macro_interp(x, xp, fp, xs, off)
