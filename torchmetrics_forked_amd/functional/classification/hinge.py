"""Hinge loss (API parity: reference ``functional/classification/hinge.py``)."""
from typing import Optional, Tuple, Union

import torch
from torch import Tensor
from typing_extensions import Literal

from torchmetrics_forked_amd.functional.classification._formats import binary_format, multiclass_format
from torchmetrics_forked_amd.functional.classification.stat_scores import (
    _binary_stat_scores_tensor_validation,
    _multiclass_stat_scores_tensor_validation,
)
from torchmetrics_forked_amd.ops import classification as cls_ops
from torchmetrics_forked_amd.utilities.data import to_onehot
from torchmetrics_forked_amd.utilities.validation import DeferredChecks
from torchmetrics_forked_amd.utilities.enums import ClassificationTaskNoMultilabel


def _hinge_loss_compute(measure: Tensor, total: Union[Tensor, int]) -> Tensor:
    return measure / total


def _binary_hinge_loss_arg_validation(squared: bool, ignore_index: Optional[int] = None) -> None:
    if not isinstance(squared, bool):
        raise ValueError(f"Expected argument `squared` to be an bool but got {squared}")
    if ignore_index is not None and not isinstance(ignore_index, int):
        raise ValueError(f"Expected argument `ignore_index` to either be `None` or an integer, but got {ignore_index}")


def _binary_hinge_loss_tensor_validation(
    preds: Tensor, target: Tensor, ignore_index: Optional[int] = None, sink: Optional[DeferredChecks] = None
) -> None:
    """``sink``: value checks become deferred device flags (GPU metric updates, no host sync)."""
    _binary_stat_scores_tensor_validation(preds, target, "global", ignore_index, sink)
    if not preds.is_floating_point():
        raise ValueError(
            "Expected argument `preds` to be floating tensor with probabilities/logits"
            f" but got tensor with dtype {preds.dtype}"
        )


def _binary_hinge_loss_update(preds: Tensor, target: Tensor, squared: bool) -> Tuple[Tensor, int]:
    margin = torch.where(target.bool(), preds, -preds)
    measures = torch.clamp(1 - margin, 0)
    if squared:
        measures = measures.pow(2)
    return measures.sum(dim=0), target.shape[0]  # host int: `total += n` needs no H2D copy


def binary_hinge_loss(
    preds: Tensor, target: Tensor, squared: bool = False, ignore_index: Optional[int] = None, validate_args: bool = False
) -> Tensor:
    if validate_args:
        _binary_hinge_loss_arg_validation(squared, ignore_index)
        _binary_hinge_loss_tensor_validation(preds, target, ignore_index)
    preds, target = binary_format(preds, target, 0.0, ignore_index, convert_to_labels=False)
    return _hinge_loss_compute(*_binary_hinge_loss_update(preds, target, squared))


def _multiclass_hinge_loss_arg_validation(
    num_classes: int, squared: bool = False, multiclass_mode: str = "crammer-singer", ignore_index: Optional[int] = None
) -> None:
    _binary_hinge_loss_arg_validation(squared, ignore_index)
    if not isinstance(num_classes, int) or num_classes < 2:
        raise ValueError(f"Expected argument `num_classes` to be an integer larger than 1, but got {num_classes}")
    allowed = ("crammer-singer", "one-vs-all")
    if multiclass_mode not in allowed:
        raise ValueError(f"Expected argument `multiclass_mode` to be one of {allowed}, but got {multiclass_mode}.")


def _multiclass_hinge_loss_tensor_validation(
    preds: Tensor, target: Tensor, num_classes: int, ignore_index: Optional[int] = None, sink: Optional[DeferredChecks] = None
) -> None:
    """``sink``: value checks become deferred device flags (GPU metric updates, no host sync)."""
    _multiclass_stat_scores_tensor_validation(preds, target, num_classes, "global", ignore_index, sink)
    if not preds.is_floating_point():
        raise ValueError(
            "Expected argument `preds` to be floating tensor with probabilities/logits"
            f" but got tensor with dtype {preds.dtype}"
        )


def _multiclass_hinge_loss_update(
    preds: Tensor, target: Tensor, squared: bool, multiclass_mode: str = "crammer-singer"
) -> Tuple[Tensor, int]:
    if preds.ndim == 2 and cls_ops.row_kernel_ok(preds, preds.shape[1]):
        # csrc/rowwise.hip: one wave per row (device softmax decision, margins, clamp, square, fixed-order sums)
        measures = cls_ops.mc_hinge(preds, target, squared, multiclass_mode != "crammer-singer").to(preds.dtype)
        return measures, preds.shape[0]
    flag = cls_ops.range_flag(preds).bool()
    preds = torch.where(flag, preds.softmax(1), preds)
    onehot = to_onehot(target, max(2, preds.shape[1])).bool()
    if multiclass_mode == "crammer-singer":
        margin = preds[onehot] - torch.max(preds.masked_fill(onehot, -float("inf")), dim=1).values
    else:
        margin = torch.where(onehot, preds, -preds)
    measures = torch.clamp(1 - margin, 0)
    if squared:
        measures = measures.pow(2)
    return measures.sum(dim=0), onehot.shape[0]


def multiclass_hinge_loss(
    preds: Tensor,
    target: Tensor,
    num_classes: int,
    squared: bool = False,
    multiclass_mode: Literal["crammer-singer", "one-vs-all"] = "crammer-singer",
    ignore_index: Optional[int] = None,
    validate_args: bool = False,
) -> Tensor:
    if validate_args:
        _multiclass_hinge_loss_arg_validation(num_classes, squared, multiclass_mode, ignore_index)
        _multiclass_hinge_loss_tensor_validation(preds, target, num_classes, ignore_index)
    preds, target = multiclass_format(preds, target, ignore_index, convert_to_labels=False)
    return _hinge_loss_compute(*_multiclass_hinge_loss_update(preds, target, squared, multiclass_mode))


def hinge_loss(
    preds: Tensor,
    target: Tensor,
    task: Literal["binary", "multiclass"],
    num_classes: Optional[int] = None,
    squared: bool = False,
    multiclass_mode: Literal["crammer-singer", "one-vs-all"] = "crammer-singer",
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    task = ClassificationTaskNoMultilabel.from_str(task)
    if task == ClassificationTaskNoMultilabel.BINARY:
        return binary_hinge_loss(preds, target, squared, ignore_index, validate_args)
    if not isinstance(num_classes, int):
        raise ValueError(f"`num_classes` is expected to be `int` but `{type(num_classes)} was passed.`")
    return multiclass_hinge_loss(preds, target, num_classes, squared, multiclass_mode, ignore_index, validate_args)
