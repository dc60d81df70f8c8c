"""Dice score (API parity: reference ``functional/classification/dice.py:24-147``), legacy auto-detected inputs."""
from typing import Optional

import torch
from torch import Tensor

from torchmetrics_forked_amd.utilities.enums import AverageMethod, MDMCAverageMethod
from torchmetrics_forked_amd.utilities.legacy_inputs import _input_squeeze, _reduce_stat_scores, _stat_scores_update


def _dice_compute(
    tp: Tensor, fp: Tensor, fn: Tensor, average: Optional[str], mdmc_average: Optional[str], zero_division: int = 0
) -> Tensor:
    numerator = 2 * tp
    denominator = 2 * tp + fp + fn
    if average == AverageMethod.MACRO and mdmc_average != MDMCAverageMethod.SAMPLEWISE:
        present = tp + fp + fn != 0
        numerator, denominator = numerator[present], denominator[present]
    if average == AverageMethod.NONE and mdmc_average != MDMCAverageMethod.SAMPLEWISE:
        absent = (tp | fn | fp) == 0
        numerator = numerator.masked_fill(absent, -1)
        denominator = denominator.masked_fill(absent, -1)
    return _reduce_stat_scores(
        numerator=numerator,
        denominator=denominator,
        weights=None if average != "weighted" else tp + fn,
        average=average,
        mdmc_average=mdmc_average,
        zero_division=zero_division,
    )


def dice(
    preds: Tensor,
    target: Tensor,
    zero_division: int = 0,
    average: Optional[str] = "micro",
    mdmc_average: Optional[str] = "global",
    threshold: float = 0.5,
    top_k: Optional[int] = None,
    num_classes: Optional[int] = None,
    multiclass: Optional[bool] = None,
    ignore_index: Optional[int] = None,
) -> Tensor:
    allowed_average = ("micro", "macro", "weighted", "samples", "none", None)
    if average not in allowed_average:
        raise ValueError(f"The `average` has to be one of {allowed_average}, got {average}.")
    if average in ("macro", "weighted", "none", None) and (not num_classes or num_classes < 1):
        raise ValueError(f"When you set `average` as {average}, you have to provide the number of classes.")
    if mdmc_average not in (None, "samplewise", "global"):
        raise ValueError(f"The `mdmc_average` has to be one of {[None, 'samplewise', 'global']}, got {mdmc_average}.")
    if num_classes and ignore_index is not None and (not ignore_index < num_classes or num_classes == 1):
        raise ValueError(f"The `ignore_index` {ignore_index} is not valid for inputs with {num_classes} classes")
    if top_k is not None and (not isinstance(top_k, int) or top_k <= 0):
        raise ValueError(f"The `top_k` should be an integer larger than 0, got {top_k}")
    preds, target = _input_squeeze(preds, target)
    reduce = "macro" if average in ("weighted", "none", None) else average
    tp, fp, _, fn = _stat_scores_update(
        preds, target, reduce=reduce, mdmc_reduce=mdmc_average, threshold=threshold, num_classes=num_classes,
        top_k=top_k, multiclass=multiclass, ignore_index=ignore_index,
    )
    return _dice_compute(tp, fp, fn, average, mdmc_average, zero_division)
