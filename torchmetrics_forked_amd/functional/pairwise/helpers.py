"""Pairwise helpers (behavioural parity: reference ``functional/pairwise/helpers.py``) + the L1/Lp dispatch to the
tiled gfx950 kernel (``csrc/pairwise.hip``)."""
from typing import Optional, Tuple

import torch
from torch import Tensor

from torchmetrics_forked_amd import ops


def _check_input(x: Tensor, y: Optional[Tensor] = None, zero_diagonal: Optional[bool] = None) -> Tuple[Tensor, Tensor, bool]:
    if x.ndim != 2:
        raise ValueError(f"Expected argument `x` to be a 2D tensor of shape `[N, d]` but got {x.shape}")
    if y is not None:
        if y.ndim != 2 or y.shape[1] != x.shape[1]:
            raise ValueError(
                "Expected argument `y` to be a 2D tensor of shape `[M, d]` where"
                " `d` should be same as the last dimension of `x`"
            )
        zero_diagonal = False if zero_diagonal is None else zero_diagonal
    else:
        y = x.clone()
        zero_diagonal = True if zero_diagonal is None else zero_diagonal
    return x, y, zero_diagonal


def _reduce_distance_matrix(distmat: Tensor, reduction: Optional[str] = None) -> Tensor:
    if reduction == "mean":
        return distmat.mean(dim=-1)
    if reduction == "sum":
        return distmat.sum(dim=-1)
    if reduction is None or reduction == "none":
        return distmat
    raise ValueError(f"Expected reduction to be one of `['mean', 'sum', None]` but got {reduction}")


def _lp_distance(x: Tensor, y: Tensor, p: float, fp64: bool) -> Tensor:
    """``[N, M]`` Lp distances; tiled HIP kernel on the GPU (no [N, M, d] intermediate), chunked eager on CPU."""
    needs_grad = torch.is_grad_enabled() and (x.requires_grad or y.requires_grad)
    if x.is_cuda and x.is_floating_point() and not needs_grad and ops.use_native(x):
        return torch.ops.tmx.pairwise_lp(x, y.to(x.dtype), float(p), fp64)
    acc = torch.float64 if fp64 else (x.dtype if x.is_floating_point() else torch.float32)
    xa, ya = x.to(acc), y.to(acc)
    rows = max(1, (1 << 26) // max(1, y.shape[0] * max(1, x.shape[1])))
    parts = []
    for s in range(0, x.shape[0], rows):
        d = (xa[s:s + rows].unsqueeze(1) - ya.unsqueeze(0)).abs()
        parts.append(d.sum(-1) if p == 1 else d.pow(p).sum(-1).pow(1.0 / p))
    return torch.cat(parts, 0) if parts else torch.empty(0, y.shape[0], dtype=acc, device=x.device)
