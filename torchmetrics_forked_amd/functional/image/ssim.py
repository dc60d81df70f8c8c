"""SSIM and multi-scale SSIM (API parity: reference ``functional/image/ssim.py:27-527``).

GPU path (4-D inputs, square window, no full-image output, no autograd): ``tmx::ssim_sums`` — a fused separable
window kernel that only visits the valid windows the reference keeps after cropping its reflect-padded conv
output, and returns per-plane sums of SSIM and contrast sensitivity (no 5·B stacked batch, no SSIM map in HBM).
Everything else follows the reference's grouped-conv formulation in PyTorch.
"""
from typing import List, Optional, Sequence, Tuple, Union

import torch
import torch.nn.functional as F
from torch import Tensor
from typing_extensions import Literal

from torchmetrics_forked_amd import ops
from torchmetrics_forked_amd.functional.image.helper import (
    _gaussian,
    _gaussian_kernel_2d,
    _gaussian_kernel_3d,
    _reflection_pad_3d,
)
from torchmetrics_forked_amd.utilities.checks import _check_same_shape
from torchmetrics_forked_amd.utilities.distributed import reduce

_NATIVE_WINDOWS = (3, 5, 7, 9, 11, 13, 15)


def _ssim_check_inputs(preds: Tensor, target: Tensor) -> Tuple[Tensor, Tensor]:
    if preds.dtype != target.dtype:
        target = target.to(preds.dtype)
    _check_same_shape(preds, target)
    if len(preds.shape) not in (4, 5):
        raise ValueError(
            "Expected `preds` and `target` to have BxCxHxW or BxCxDxHxW shape."
            f" Got preds: {preds.shape} and target: {target.shape}."
        )
    return preds, target


def _data_range_and_clamp(
    preds: Tensor, target: Tensor, data_range: Optional[Union[float, Tuple[float, float]]]
) -> Tuple[Tensor, Tensor, Union[float, Tensor]]:
    if data_range is None:
        return preds, target, torch.maximum(preds.max() - preds.min(), target.max() - target.min())
    if isinstance(data_range, tuple):
        preds = torch.clamp(preds, min=data_range[0], max=data_range[1])
        target = torch.clamp(target, min=data_range[0], max=data_range[1])
        return preds, target, data_range[1] - data_range[0]
    return preds, target, data_range


def _native_ssim_ok(preds: Tensor, window: Sequence[int], return_full_image: bool) -> bool:
    if not preds.is_cuda or preds.ndim != 4 or return_full_image:
        return False
    if torch.is_grad_enabled() and preds.requires_grad:
        return False
    if window[0] != window[1] or window[0] not in _NATIVE_WINDOWS:
        return False
    h, w = preds.shape[-2:]
    return h >= window[0] and w >= window[1] and ops.use_native(preds)


def _ssim_update(
    preds: Tensor,
    target: Tensor,
    gaussian_kernel: bool = True,
    sigma: Union[float, Sequence[float]] = 1.5,
    kernel_size: Union[int, Sequence[int]] = 11,
    data_range: Optional[Union[float, Tuple[float, float]]] = None,
    k1: float = 0.01,
    k2: float = 0.03,
    return_full_image: bool = False,
    return_contrast_sensitivity: bool = False,
    sse_out: Optional[List[Tensor]] = None,
) -> Union[Tensor, Tuple[Tensor, Tensor]]:
    """Per-image SSIM ``[B]`` (optionally with per-image contrast sensitivity or the full SSIM map).

    ``sse_out``: when the native kernel runs, the total squared error of the batch (fp64) is appended to it — the
    kernel accumulates it while staging the pixels (fused PSNR of a ``MetricCollection``, ``ops/fused.py``)."""
    is_3d = preds.ndim == 5
    if not isinstance(kernel_size, Sequence):
        kernel_size = 3 * [kernel_size] if is_3d else 2 * [kernel_size]
    if not isinstance(sigma, Sequence):
        sigma = 3 * [sigma] if is_3d else 2 * [sigma]
    if len(kernel_size) != len(target.shape) - 2:
        raise ValueError(
            f"`kernel_size` has dimension {len(kernel_size)}, but expected to be two less that target dimensionality,"
            f" which is: {len(target.shape)}"
        )
    if len(kernel_size) not in (2, 3):
        raise ValueError(f"Expected `kernel_size` dimension to be 2 or 3. `kernel_size` dimensionality: {len(kernel_size)}")
    if len(sigma) != len(target.shape) - 2:
        raise ValueError(
            f"`kernel_size` has dimension {len(kernel_size)}, but expected to be two less that target dimensionality,"
            f" which is: {len(target.shape)}"
        )
    if len(sigma) not in (2, 3):
        raise ValueError(f"Expected `kernel_size` dimension to be 2 or 3. `kernel_size` dimensionality: {len(kernel_size)}")
    if return_full_image and return_contrast_sensitivity:
        raise ValueError("Arguments `return_full_image` and `return_contrast_sensitivity` are mutually exclusive.")
    if any(x % 2 == 0 or x <= 0 for x in kernel_size):
        raise ValueError(f"Expected `kernel_size` to have odd positive number. Got {kernel_size}.")
    if any(y <= 0 for y in sigma):
        raise ValueError(f"Expected `sigma` to have positive number. Got {sigma}.")

    preds, target, data_range = _data_range_and_clamp(preds, target, data_range)
    c1 = (k1 * data_range) ** 2
    c2 = (k2 * data_range) ** 2
    channel, dtype, device = preds.size(1), preds.dtype, preds.device
    gks = [int(3.5 * s + 0.5) * 2 + 1 for s in sigma]
    window = gks if gaussian_kernel else list(kernel_size)

    if not is_3d and _native_ssim_ok(preds, window, return_full_image) and (gaussian_kernel is False or sigma[0] == sigma[1]):
        if gaussian_kernel:
            w1 = _gaussian(gks[0], sigma[0], torch.float32, device).reshape(-1)
        else:
            w1 = torch.full((window[0],), 1.0 / window[0], dtype=torch.float32, device=device)
        # fill kernels for Python-float constants (a pageable host-to-device copy would block the host)
        # (c1, c2, data range): the range sets the matrix-core kernel's exact power-of-two operand scaling
        consts = torch.stack([c.to(device, torch.float32) if isinstance(c, torch.Tensor) else torch.full((), float(c), device=device)
                              for c in (c1, c2, data_range)])
        b, c, h, w = preds.shape
        sums = torch.ops.tmx.ssim_sums(preds.reshape(b * c, h, w), target.reshape(b * c, h, w), w1, w1, consts, sse_out is not None)
        if sse_out is not None:
            sse_out.append(sums[2].sum())
        n_valid = c * (h - window[0] + 1) * (w - window[1] + 1)
        sim = (sums[0].reshape(b, c).sum(1) / n_valid).to(dtype)
        if return_contrast_sensitivity:
            return sim, (sums[1].reshape(b, c).sum(1) / n_valid).to(dtype)
        return sim

    pad_h = (gks[0] - 1) // 2
    pad_w = (gks[1] - 1) // 2
    if is_3d:
        pad_d = (gks[2] - 1) // 2
        preds = _reflection_pad_3d(preds, pad_d, pad_w, pad_h)
        target = _reflection_pad_3d(target, pad_d, pad_w, pad_h)
        kernel = _gaussian_kernel_3d(channel, gks, sigma, dtype, device) if gaussian_kernel else None
    else:
        preds = F.pad(preds, (pad_w, pad_w, pad_h, pad_h), mode="reflect")
        target = F.pad(target, (pad_w, pad_w, pad_h, pad_h), mode="reflect")
        kernel = _gaussian_kernel_2d(channel, gks, sigma, dtype, device) if gaussian_kernel else None
    if not gaussian_kernel:
        kernel = torch.ones((channel, 1, *kernel_size), dtype=dtype, device=device) / torch.prod(
            torch.tensor(kernel_size, dtype=dtype, device=device)
        )
    stacked = torch.cat((preds, target, preds * preds, target * target, preds * target))
    outputs = F.conv3d(stacked, kernel, groups=channel) if is_3d else F.conv2d(stacked, kernel, groups=channel)
    mu_p, mu_t, e_pp, e_tt, e_pt = outputs.split(preds.shape[0])
    mu_pp, mu_tt, mu_pt = mu_p.pow(2), mu_t.pow(2), mu_p * mu_t
    upper = 2 * (e_pt - mu_pt).to(dtype) + c2
    lower = ((e_pp - mu_pp) + (e_tt - mu_tt)).to(dtype) + c2
    full = ((2 * mu_pt + c1) * upper) / ((mu_pp + mu_tt + c1) * lower)
    crop = (slice(pad_h, -pad_h), slice(pad_w, -pad_w), slice(pad_d, -pad_d)) if is_3d else (slice(pad_h, -pad_h), slice(pad_w, -pad_w))
    ssim_idx = full[(..., *crop)]
    per_image = ssim_idx.reshape(ssim_idx.shape[0], -1).mean(-1)
    if return_contrast_sensitivity:
        cs = (upper / lower)[(..., *crop)]
        return per_image, cs.reshape(cs.shape[0], -1).mean(-1)
    if return_full_image:
        return per_image, full
    return per_image


def _ssim_compute(similarities: Tensor, reduction: Literal["elementwise_mean", "sum", "none", None] = "elementwise_mean") -> Tensor:
    return reduce(similarities, reduction)


def structural_similarity_index_measure(
    preds: Tensor,
    target: Tensor,
    gaussian_kernel: bool = True,
    sigma: Union[float, Sequence[float]] = 1.5,
    kernel_size: Union[int, Sequence[int]] = 11,
    reduction: Literal["elementwise_mean", "sum", "none", None] = "elementwise_mean",
    data_range: Optional[Union[float, Tuple[float, float]]] = None,
    k1: float = 0.01,
    k2: float = 0.03,
    return_full_image: bool = False,
    return_contrast_sensitivity: bool = False,
) -> Union[Tensor, Tuple[Tensor, Tensor]]:
    preds, target = _ssim_check_inputs(preds, target)
    pack = _ssim_update(preds, target, gaussian_kernel, sigma, kernel_size, data_range, k1, k2, return_full_image,
                        return_contrast_sensitivity)
    if isinstance(pack, tuple):
        return _ssim_compute(pack[0], reduction), pack[1]
    return _ssim_compute(pack, reduction)


def _get_normalized_sim_and_cs(
    preds: Tensor,
    target: Tensor,
    gaussian_kernel: bool = True,
    sigma: Union[float, Sequence[float]] = 1.5,
    kernel_size: Union[int, Sequence[int]] = 11,
    data_range: Optional[Union[float, Tuple[float, float]]] = None,
    k1: float = 0.01,
    k2: float = 0.03,
    normalize: Optional[Literal["relu", "simple"]] = None,
) -> Tuple[Tensor, Tensor]:
    sim, cs = _ssim_update(preds, target, gaussian_kernel, sigma, kernel_size, data_range, k1, k2, return_contrast_sensitivity=True)
    if normalize == "relu":
        sim, cs = torch.relu(sim), torch.relu(cs)
    return sim, cs


def _multiscale_ssim_update(
    preds: Tensor,
    target: Tensor,
    gaussian_kernel: bool = True,
    sigma: Union[float, Sequence[float]] = 1.5,
    kernel_size: Union[int, Sequence[int]] = 11,
    data_range: Optional[Union[float, Tuple[float, float]]] = None,
    k1: float = 0.01,
    k2: float = 0.03,
    betas: Tuple[float, ...] = (0.0448, 0.2856, 0.3001, 0.2363, 0.1333),
    normalize: Optional[Literal["relu", "simple"]] = None,
) -> Tensor:
    mcs_list: List[Tensor] = []
    is_3d = preds.ndim == 5
    if not isinstance(kernel_size, Sequence):
        kernel_size = 3 * [kernel_size] if is_3d else 2 * [kernel_size]
    if not isinstance(sigma, Sequence):
        sigma = 3 * [sigma] if is_3d else 2 * [sigma]
    if preds.size()[-1] < 2 ** len(betas) or preds.size()[-2] < 2 ** len(betas):
        raise ValueError(
            f"For a given number of `betas` parameters {len(betas)}, the image height and width dimensions must be"
            f" larger than or equal to {2 ** len(betas)}."
        )
    div = max(1, len(betas) - 1) ** 2
    if preds.size()[-2] // div <= kernel_size[0] - 1:
        raise ValueError(
            f"For a given number of `betas` parameters {len(betas)} and kernel size {kernel_size[0]},"
            f" the image height must be larger than {(kernel_size[0] - 1) * div}."
        )
    if preds.size()[-1] // div <= kernel_size[1] - 1:
        raise ValueError(
            f"For a given number of `betas` parameters {len(betas)} and kernel size {kernel_size[1]},"
            f" the image width must be larger than {(kernel_size[1] - 1) * div}."
        )
    sim = None
    for _ in range(len(betas)):
        sim, cs = _get_normalized_sim_and_cs(preds, target, gaussian_kernel, sigma, kernel_size, data_range, k1, k2, normalize=normalize)
        mcs_list.append(cs)
        if len(kernel_size) == 2:
            preds, target = F.avg_pool2d(preds, (2, 2)), F.avg_pool2d(target, (2, 2))
        else:
            preds, target = F.avg_pool3d(preds, (2, 2, 2)), F.avg_pool3d(target, (2, 2, 2))
    mcs_list[-1] = sim
    stack = torch.stack(mcs_list)
    if normalize == "simple":
        stack = (stack + 1) / 2
    betas_t = torch.tensor(betas, device=stack.device).view(-1, 1)
    return torch.prod(stack**betas_t, dim=0)


def _multiscale_ssim_compute(mcs_per_image: Tensor, reduction: Literal["elementwise_mean", "sum", "none", None] = "elementwise_mean") -> Tensor:
    return reduce(mcs_per_image, reduction)


def multiscale_structural_similarity_index_measure(
    preds: Tensor,
    target: Tensor,
    gaussian_kernel: bool = True,
    sigma: Union[float, Sequence[float]] = 1.5,
    kernel_size: Union[int, Sequence[int]] = 11,
    reduction: Literal["elementwise_mean", "sum", "none", None] = "elementwise_mean",
    data_range: Optional[Union[float, Tuple[float, float]]] = None,
    k1: float = 0.01,
    k2: float = 0.03,
    betas: Tuple[float, ...] = (0.0448, 0.2856, 0.3001, 0.2363, 0.1333),
    normalize: Optional[Literal["relu", "simple"]] = "relu",
) -> Tensor:
    if not isinstance(betas, tuple):
        raise ValueError("Argument `betas` is expected to be of a type tuple.")
    if isinstance(betas, tuple) and not all(isinstance(beta, float) for beta in betas):
        raise ValueError("Argument `betas` is expected to be a tuple of floats.")
    if normalize and normalize not in ("relu", "simple"):
        raise ValueError("Argument `normalize` to be expected either `None` or one of 'relu' or 'simple'")
    preds, target = _ssim_check_inputs(preds, target)
    mcs = _multiscale_ssim_update(preds, target, gaussian_kernel, sigma, kernel_size, data_range, k1, k2, betas, normalize)
    return _multiscale_ssim_compute(mcs, reduction)
