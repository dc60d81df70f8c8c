"""Pairwise helpers (behavioural parity: reference ``functional/pairwise/helpers.py``) + the L1/Lp dispatch to the
tiled gfx950 kernel (``csrc/pairwise.hip``)."""
from typing import Optional, Tuple

import torch
from torch import Tensor

from torchmetrics_forked_amd import ops


def _check_input(x: Tensor, y: Optional[Tensor] = None, zero_diagonal: Optional[bool] = None, clone: bool = True) -> Tuple[Tensor, Tensor, bool]:
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
        y = x.clone() if clone else x
        zero_diagonal = True if zero_diagonal is None else zero_diagonal
    return x, y, zero_diagonal


_GEMM_MODES = {"linear": 0, "cosine": 1, "euclidean": 2}
_FUSED = True  # False: always the ATen composition; "force": always the kernel (tests, tools/pairwise_bench.py)


def _fused_wins(mode: str, dtype: torch.dtype, n: int, m: int, d: int) -> bool:
    """Measured routing (``tools/pairwise_bench.py``, ``profiles/pairwise_gemm_r5.json``; work = n * m * d).
    Euclidean: the kernel keeps the reference's fp64 N x M chain (five HBM round trips) out of memory and wins at every
    measured shape up to d = 1024 (1.05-4.2x); deeper, rocBLAS's dgemm out-runs the kernel's fp64 MFMA loop.  Linear / cosine are a plain library GEMM plus a diagonal fill / row normalisation: the
    kernel wins while the launches dominate, hipBLASLt beyond.  16-bit inputs with at least 256 128 x 128 output tiles
    run on the kernel's bf16 / fp16 MFMA tiles (1.0-3.3x over hipBLASLt + the epilogue up to 2^33 work and 2^25
    outputs); smaller outputs take its fp32 MFMA tiles, which win only while the launches dominate.  fp32 with at least
    256 128 x 128 tiles runs on the f16-split matrix-core route at every depth."""
    work = n * m * d
    if mode == "euclidean":
        return d <= 1024 or work <= (1 << 31)
    if dtype == torch.float64:  # rocBLAS's dgemm beats the fp64 MFMA loop on the plain product
        return mode == "cosine" and work <= (1 << 29) and d <= 256
    if dtype in (torch.bfloat16, torch.float16):
        if ((n + 127) // 128) * ((m + 127) // 128) >= 256:  # the kernel's 16-bit MFMA tiles (csrc: kPhT)
            return work <= (1 << 33) and n * m <= (1 << 25)
        return work <= (1 << 29) and d <= (256 if mode == "linear" else 1024)
    if ((n + 127) // 128) * ((m + 127) // 128) >= 256:
        # fp32 on f16 matrix cores (csrc/pairwise.hip x3: two-plane split, three products): 1.45-2.4x over hipBLASLt's
        # fp32 GEMM from 2048^2 x 2048 to 10,000^2 x 2048 (profiles/pairwise_gemm_r6.json)
        return True
    return work < (1 << 32) and d <= (512 if mode == "linear" else 1024)


def _native_gemm(x: Tensor, y: Optional[Tensor], mode: str, zero_diagonal: Optional[bool]) -> Optional[Tensor]:
    """The GEMM forms as one fused MFMA kernel (``csrc/pairwise.hip`` ``pairwise_gemm``: dot products, norms and the
    epilogue in one pass, the input dtype written once) for GPU float inputs of one dtype without autograd; ``None``
    sends the caller down the ATen composition (reference ``functional/pairwise/{linear,cosine,euclidean}.py``)."""
    if not (_FUSED and isinstance(x, Tensor) and x.is_cuda and x.is_floating_point()):
        return None
    if y is not None and (y.dtype != x.dtype or y.device != x.device):
        return None
    if torch.is_grad_enabled() and (x.requires_grad or (y is not None and y.requires_grad)):
        return None
    if not ops.use_native(x):
        return None
    x, y, zero_diagonal = _check_input(x, y, zero_diagonal, clone=False)
    if x.shape[1] == 0:
        return None
    if _FUSED != "force" and not _fused_wins(mode, x.dtype, x.shape[0], y.shape[0], x.shape[1]):
        return None
    return torch.ops.tmx.pairwise_gemm(x, y, _GEMM_MODES[mode], bool(zero_diagonal))


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
