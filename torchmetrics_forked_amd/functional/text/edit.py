"""Levenshtein edit distance with substitution cost (API parity: reference ``functional/text/edit.py``).

Scores come from the native Tercom-style beam DP (``tmx::levenshtein_beam_batch``), which is what the reference
evaluates (``_LevenshteinEditDistance``: beam of 25 around the length-ratio diagonal, insertion = deletion = 1)."""
from typing import Literal, Optional, Sequence, Union

import torch
from torch import Tensor

from torchmetrics_forked_amd import ops
from torchmetrics_forked_amd.functional.text.helper import _pack_codepoints


# characters (reference side) above which a GPU-resident metric runs the pair DPs on the device
GPU_EDIT_MIN_CHARS = 2048


def _edit_distance_update(
    preds: Union[str, Sequence[str]],
    target: Union[str, Sequence[str]],
    substitution_cost: int = 1,
    device: Optional[torch.device] = None,
) -> Tensor:
    """Per-pair distances.  With ``device`` on the GPU (a GPU-resident ``EditDistance``) and enough text, the beam DPs
    run there (``tmx::levenshtein_beam_gpu``, one thread per pair, identical integers) and the scores stay on the
    device; otherwise the host op."""
    if isinstance(preds, str):
        preds = [preds]
    if isinstance(target, str):
        target = [target]
    if not all(isinstance(x, str) for x in preds):
        raise ValueError(f"Expected all values in argument `preds` to be string type, but got {preds}")
    if not all(isinstance(x, str) for x in target):
        raise ValueError(f"Expected all values in argument `target` to be string type, but got {target}")
    if len(preds) != len(target):
        raise ValueError(
            f"Expected argument `preds` and `target` to have same length, but got {len(preds)} and {len(target)}"
        )
    ops.require()
    p, p_off = _pack_codepoints(preds)
    t, t_off = _pack_codepoints(target)
    max_ref = max((len(x) for x in target), default=0)
    if (device is not None and device.type == "cuda" and t.numel() >= GPU_EDIT_MIN_CHARS
            and (max_ref + 1) * len(target) * 8 <= (1 << 30)  # one int64 DP row per pair in the scratch
            and ops.use_native(torch.empty(0, device=device))):
        d = [x.to(device, non_blocking=True) for x in (p, p_off, t, t_off)]
        return torch.ops.tmx.levenshtein_beam_gpu(*d, 1, 1, int(substitution_cost), max_ref).int()
    return torch.ops.tmx.levenshtein_beam_batch(p, p_off, t, t_off, 1, 1, int(substitution_cost)).int()


def _edit_distance_compute(
    edit_scores: Tensor,
    num_elements: Union[Tensor, int],
    reduction: Optional[Literal["mean", "sum", "none"]] = "mean",
) -> Tensor:
    if edit_scores.numel() == 0:
        return torch.tensor(0, dtype=torch.int32)
    if reduction == "mean":
        return edit_scores.sum() / num_elements
    if reduction == "sum":
        return edit_scores.sum()
    if reduction is None or reduction == "none":
        return edit_scores
    raise ValueError("Expected argument `reduction` to either be 'sum', 'mean', 'none' or None")


def edit_distance(
    preds: Union[str, Sequence[str]],
    target: Union[str, Sequence[str]],
    substitution_cost: int = 1,
    reduction: Optional[Literal["mean", "sum", "none"]] = "mean",
) -> Tensor:
    """Character-level edit distance between each prediction and its target."""
    distance = _edit_distance_update(preds, target, substitution_cost)
    return _edit_distance_compute(distance, num_elements=distance.numel(), reduction=reduction)
