"""Python entry point for the regression map-reduce kernel (``csrc/regression.hip``).

``regression_sums(preds, target, op, param)`` returns the fp64 ``[8, D]`` table
``(Σp, Σt, Σp², Σt², Σpt, Σ(p−t)², Σ|p−t|, Σ op(p,t))`` of a ``[N, D]`` input pair in ONE pass.  On GPU tensors the
native kernel is mandatory; the eager implementation below is the CPU path and the numerics oracle of the GPU
tests.  Callers use the fused path only when no autograd graph is needed (``fused_ok``), so differentiable
functional calls keep exact PyTorch semantics.
"""
from typing import Optional, List

import torch
from torch import Tensor

from torchmetrics_forked_amd import ops

OP_NONE, OP_APE, OP_SAPE, OP_SLE, OP_LOGCOSH, OP_MINKOWSKI, OP_ABS_T, OP_TWEEDIE = range(8)
_EPS = 1.17e-06


def fused_ok(*tensors: Tensor) -> bool:
    """True when the fused kernel may be used: GPU tensors, float dtype, no autograd recording."""
    t0 = tensors[0]
    if not t0.is_cuda:
        return False
    if torch.is_grad_enabled() and any(t.requires_grad for t in tensors):
        return False
    return all(t.is_floating_point() for t in tensors) and ops.use_native(t0)


def _eager_op(op: int, p: Tensor, t: Tensor, param: float) -> Tensor:
    d = p - t
    if op == OP_APE:
        return d.abs() / t.abs().clamp(min=_EPS)
    if op == OP_SAPE:
        return 2 * (d.abs() / (t.abs() + p.abs()).clamp(min=_EPS))
    if op == OP_SLE:
        return (torch.log1p(p) - torch.log1p(t)) ** 2
    if op == OP_LOGCOSH:
        return torch.log((torch.exp(d) + torch.exp(-d)) / 2)
    if op == OP_MINKOWSKI:
        return d.abs().pow(param)
    if op == OP_ABS_T:
        return t.abs()
    if op == OP_TWEEDIE:
        if param == 0:
            return (t - p) ** 2
        if param == 1:
            return 2 * (torch.xlogy(t, t / p) + p - t)
        if param == 2:
            return 2 * (torch.log(p / t) + t / p - 1)
        term1 = torch.clamp(t, min=0).pow(2 - param) / ((1 - param) * (2 - param))
        term2 = t * p.pow(1 - param) / (1 - param)
        term3 = p.pow(2 - param) / (2 - param)
        return 2 * (term1 - term2 + term3)
    return torch.zeros_like(p)


def regression_sums(preds: Tensor, target: Tensor, op: int = OP_NONE, param: float = 0.0) -> Tensor:
    if preds.ndim == 1:
        preds, target = preds.unsqueeze(1), target.unsqueeze(1)
    if preds.dtype != target.dtype:
        dt = torch.promote_types(preds.dtype, target.dtype)
        preds, target = preds.to(dt), target.to(dt)
    if ops.use_native(preds):
        return torch.ops.tmx.regression_sums(preds, target, int(op), float(param))
    cdt = torch.float64 if preds.dtype == torch.float64 else torch.float32
    p, t = preds.to(cdt), target.to(cdt)
    d = p - t
    chans = [p, t, p * p, t * t, p * t, d * d, d.abs(), _eager_op(op, p, t, param)]
    return torch.stack([c.double().sum(0) for c in chans])


CH_SQ, CH_ABS = 5, 6  # channels of regression_sums: sum of squared / absolute differences


def accumulate(preds: Tensor, target: Tensor, op: int, param: float, chans: List[int], states: List[Tensor], total: Optional[Tensor],
               n_add: int) -> bool:
    """``states[i] += sums[chans[i]]`` (cast to the inputs' dtype, as the eager update) and ``total += n_add`` in place,
    one map-reduce launch + one tiny fold launch (csrc/regression.hip ``regression_accumulate``).  ``preds`` /
    ``target``: ``[N]`` or ``[N, D]``.  Returns False (nothing done) when the eager path must run: CPU, autograd,
    16-bit or mixed input dtypes, or states that are not contiguous float32 / float64 ``[D]`` on the inputs' device."""
    if not fused_ok(preds, target) or preds.dtype != target.dtype or preds.dtype not in (torch.float32, torch.float64):
        return False
    if preds.ndim == 1:
        preds, target = preds.unsqueeze(1), target.unsqueeze(1)
    elif preds.ndim != 2:
        return False
    dev, D = preds.device, preds.shape[1]
    for st in states:
        if st.device != dev or not st.is_contiguous() or st.numel() != D or st.dtype not in (torch.float32, torch.float64):
            return False
    if total is not None and (total.device != dev or total.dtype != torch.long or total.numel() != 1):
        return False
    torch.ops.tmx.regression_accumulate(preds, target, int(op), float(param), list(chans), list(states), total, int(n_add))
    return True
