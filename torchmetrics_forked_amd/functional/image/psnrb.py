"""PSNR with blocking-effect factor (API parity: reference ``functional/image/psnrb.py:22-130``).

The blocking-effect sums use strided slices of the boundary / non-boundary column and row differences instead
of host-built index lists."""
import math
from typing import Tuple

import torch
from torch import Tensor, tensor


def _compute_bef(x: Tensor, block_size: int = 8) -> Tensor:
    _, channels, height, width = x.shape
    if channels > 1:
        raise ValueError(f"`psnrb` metric expects grayscale images, but got images with {channels} channels.")
    dh = (x[..., :, :-1] - x[..., :, 1:]).pow(2.0)  # [.., H, W-1]: difference at column boundary j|j+1
    dv = (x[..., :-1, :] - x[..., 1:, :]).pow(2.0)
    hb = torch.zeros(width - 1, dtype=torch.bool, device=x.device)
    hb[block_size - 1 :: block_size] = True
    vb = torch.zeros(height - 1, dtype=torch.bool, device=x.device)
    vb[block_size - 1 :: block_size] = True
    d_b = dh[..., hb].sum() + dv[..., vb, :].sum()
    d_bc = dh[..., ~hb].sum() + dv[..., ~vb, :].sum()
    n_hb = height * (width / block_size) - 1
    n_hbc = height * (width - 1) - n_hb
    n_vb = width * (height / block_size) - 1
    n_vbc = width * (height - 1) - n_vb
    d_b = d_b / (n_hb + n_vb)
    d_bc = d_bc / (n_hbc + n_vbc)
    t = math.log2(block_size) / math.log2(min(height, width)) if d_b > d_bc else 0
    return t * (d_b - d_bc)


def _psnrb_compute(sum_squared_error: Tensor, bef: Tensor, num_obs: Tensor, data_range: Tensor) -> Tensor:
    mse = sum_squared_error / num_obs + bef
    if data_range > 2:
        return 10 * torch.log10(data_range**2 / mse)
    return 10 * torch.log10(1.0 / mse)


def _psnrb_update(preds: Tensor, target: Tensor, block_size: int = 8) -> Tuple[Tensor, Tensor, Tensor]:
    sse = torch.sum(torch.pow(preds - target, 2))
    return sse, _compute_bef(preds, block_size=block_size), tensor(target.numel(), device=target.device)


def peak_signal_noise_ratio_with_blocked_effect(preds: Tensor, target: Tensor, block_size: int = 8) -> Tensor:
    data_range = target.max() - target.min()
    sse, bef, n = _psnrb_update(preds, target, block_size=block_size)
    return _psnrb_compute(sse, bef, n, data_range)
