"""Perplexity (API parity: reference ``functional/text/perplexity.py``).

GPU inputs run the fused token-NLL kernel ``tmx::token_nll`` (one streaming pass over the logits, online
log-sum-exp, direct target gather); CPU / autograd inputs use ``log_softmax`` + ``gather``.  Both replace the
reference's ``softmax`` + ``[N, N]`` diagonal gather (same value up to floating-point rounding, no quadratic
memory, and log-softmax avoids ``log(0)`` for vanishing probabilities)."""
from typing import Optional, Tuple

import torch
from torch import Tensor

from torchmetrics_forked_amd import ops

_TORCH_FLOAT_OR_DOUBLE = (torch.float32, torch.float64)


def _check_shape_and_type_consistency(preds: Tensor, target: Tensor) -> None:
    if len(preds.shape) != 3:
        raise ValueError(
            "Input tensor `preds` is expected to have 3 dimensions, [batch_size, seq_len, vocab_size],"
            f" but got {len(preds.shape)}."
        )
    if len(target.shape) != 2:
        raise ValueError(
            "Input tensor `target` is expected to have 2 dimensions, [batch_size, seq_len],"
            f" but got {len(target.shape)}."
        )
    if preds.shape[:2] != target.shape:
        raise ValueError(
            "Input tensors `preds` and `target` are expected to have equaling first two dimensions,"
            f" [batch_size, seq_len], but got {preds.shape[:2]} and {target.shape}."
        )
    if preds.dtype not in _TORCH_FLOAT_OR_DOUBLE:
        raise TypeError(
            f"Input tensor `preds` is expected to be of a type one of {_TORCH_FLOAT_OR_DOUBLE} but got {preds.dtype}."
        )
    if target.dtype != torch.int64:
        raise TypeError(f"Input tensor `target` is expected to be of a type {torch.int64} but got {target.dtype}.")


def _perplexity_update(preds: Tensor, target: Tensor, ignore_index: Optional[int] = None) -> Tuple[Tensor, Tensor]:
    _check_shape_and_type_consistency(preds, target)
    logits = preds.reshape(-1, preds.shape[-1])
    tgt = target.reshape(-1)
    mask = tgt.ne(ignore_index) if ignore_index is not None else torch.ones_like(tgt, dtype=torch.bool)
    grad = torch.is_grad_enabled() and preds.requires_grad
    if not grad and ops.use_native(logits):
        nll = torch.ops.tmx.token_nll(logits, tgt, int(ignore_index) if ignore_index is not None else 0, ignore_index is not None)
        total = nll.double().sum().to(preds.dtype)
    else:
        safe = torch.where(mask, tgt, torch.zeros_like(tgt))
        logp = torch.log_softmax(logits, dim=1).gather(1, safe[:, None]).squeeze(1)
        total = -(logp[mask]).sum()
    return total, mask.sum()


def _perplexity_compute(total: Tensor, count: Tensor) -> Tensor:
    return torch.exp(total / count)


def perplexity(preds: Tensor, target: Tensor, ignore_index: Optional[int] = None) -> Tensor:
    """exp(mean token negative log-likelihood) of ``target`` under the logits ``preds`` ``[B, S, V]``."""
    total, count = _perplexity_update(preds, target, ignore_index)
    return _perplexity_compute(total, count)
