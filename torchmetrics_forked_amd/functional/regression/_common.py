"""Shared regression helpers (reference ``functional/regression/utils.py``) and the fused-sums dispatch."""
from typing import Optional

import torch
from torch import Tensor

from torchmetrics_forked_amd.ops import regression as reg_ops


def _check_data_shape_to_num_outputs(preds: Tensor, target: Tensor, num_outputs: int, allow_1d_reshape: bool = False) -> None:
    if preds.ndim > 2 or target.ndim > 2:
        raise ValueError(
            "Expected both predictions and target to be either 1- or 2-dimensional tensors,"
            f" but got {target.ndim} and {preds.ndim}."
        )
    cond1 = not allow_1d_reshape and num_outputs == 1 and not (preds.ndim == 1 or preds.shape[1] == 1)
    cond2 = num_outputs > 1 and preds.ndim > 1 and num_outputs != preds.shape[1]
    if cond1 or cond2:
        raise ValueError(
            "Expected argument `num_outputs` to match the second dimension of input, but got"
            f" {num_outputs} and {preds.shape[1]}."
        )


def fused_sums(preds: Tensor, target: Tensor, op: int = reg_ops.OP_NONE, param: float = 0.0, flatten: bool = False) -> Optional[Tensor]:
    """fp64 ``[8, D]`` sums from the HIP kernel, or ``None`` when the eager (autograd / CPU) path must run."""
    if not reg_ops.fused_ok(preds, target):
        return None
    if flatten:
        preds, target = preds.reshape(-1), target.reshape(-1)
    return reg_ops.regression_sums(preds, target, op, param)


def _out_dtype(preds: Tensor, target: Tensor) -> torch.dtype:
    dt = torch.promote_types(preds.dtype, target.dtype)
    return dt if dt.is_floating_point else torch.get_default_dtype()
