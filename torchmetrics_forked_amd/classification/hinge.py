"""Hinge-loss modules (API parity: reference ``classification/hinge.py:41-355``)."""
from typing import Any, Optional, Type

import torch
from torch import Tensor
from typing_extensions import Literal

from torchmetrics_forked_amd.classification.base import _ClassificationTaskWrapper
from torchmetrics_forked_amd.functional.classification._formats import binary_format, multiclass_format
from torchmetrics_forked_amd.functional.classification.hinge import (
    _binary_hinge_loss_arg_validation,
    _binary_hinge_loss_tensor_validation,
    _binary_hinge_loss_update,
    _hinge_loss_compute,
    _multiclass_hinge_loss_arg_validation,
    _multiclass_hinge_loss_tensor_validation,
    _multiclass_hinge_loss_update,
)
from torchmetrics_forked_amd.metric import Metric
from torchmetrics_forked_amd.utilities.enums import ClassificationTaskNoMultilabel
from torchmetrics_forked_amd.utilities.plot import _AX_TYPE, _PLOT_OUT_TYPE


class _HingeBase(Metric):
    is_differentiable: bool = True
    higher_is_better: bool = False
    full_state_update: bool = False
    plot_lower_bound: float = 0.0
    measures: Tensor
    total: Tensor

    def compute(self) -> Tensor:
        return _hinge_loss_compute(self.measures, self.total)

    def plot(self, val: Optional[Tensor] = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:
        return self._plot(val, ax)


class BinaryHingeLoss(_HingeBase):
    """BinaryHingeLoss (binary task).

    Example:
        >>> import torch
        >>> from torchmetrics_forked_amd.classification import BinaryHingeLoss
        >>> preds = torch.tensor([0.1, 0.8, 0.6, 0.3, 0.9, 0.2])
        >>> target = torch.tensor([0, 1, 0, 0, 1, 1])
        >>> metric = BinaryHingeLoss()
        >>> metric(preds, target)
        tensor(0.8500)
    """
    def __init__(
        self, squared: bool = False, ignore_index: Optional[int] = None, validate_args: bool = True, **kwargs: Any
    ) -> None:
        super().__init__(**kwargs)
        if validate_args:
            _binary_hinge_loss_arg_validation(squared, ignore_index)
        self.validate_args = validate_args
        self.squared = squared
        self.ignore_index = ignore_index
        self.add_state("measures", default=torch.tensor(0.0), dist_reduce_fx="sum")
        self.add_state("total", default=torch.tensor(0), dist_reduce_fx="sum")

    def update(self, preds: Tensor, target: Tensor) -> None:
        if self.validate_args:
            _binary_hinge_loss_tensor_validation(preds, target, self.ignore_index, self._validation_sink(target))
        preds, target = binary_format(preds, target, 0.0, self.ignore_index, convert_to_labels=False)
        measures, total = _binary_hinge_loss_update(preds, target, self.squared)
        self.measures += measures
        self.total += total


class MulticlassHingeLoss(_HingeBase):
    """Multiclass hinge loss (crammer-singer or one-vs-all).

    Example:
        >>> import torch
        >>> from torchmetrics_forked_amd.classification import MulticlassHingeLoss
        >>> preds = torch.tensor([[0.25, 0.20, 0.55], [0.55, 0.05, 0.40], [0.10, 0.30, 0.60], [0.90, 0.05, 0.05]])
        >>> MulticlassHingeLoss(num_classes=3)(preds, torch.tensor([0, 1, 2, 0]))
        tensor(0.9125)
        >>> MulticlassHingeLoss(num_classes=3, multiclass_mode='one-vs-all')(preds, torch.tensor([0, 1, 2, 0]))
        tensor([0.8750, 1.1250, 1.1000])
    """
    def __init__(
        self,
        num_classes: int,
        squared: bool = False,
        multiclass_mode: Literal["crammer-singer", "one-vs-all"] = "crammer-singer",
        ignore_index: Optional[int] = None,
        validate_args: bool = True,
        **kwargs: Any,
    ) -> None:
        super().__init__(**kwargs)
        if validate_args:
            _multiclass_hinge_loss_arg_validation(num_classes, squared, multiclass_mode, ignore_index)
        self.validate_args = validate_args
        self.num_classes = num_classes
        self.squared = squared
        self.multiclass_mode = multiclass_mode
        self.ignore_index = ignore_index
        default = torch.tensor(0.0) if multiclass_mode == "crammer-singer" else torch.zeros(num_classes)
        self.add_state("measures", default=default, dist_reduce_fx="sum")
        self.add_state("total", default=torch.tensor(0), dist_reduce_fx="sum")

    def update(self, preds: Tensor, target: Tensor) -> None:
        if self.validate_args:
            _multiclass_hinge_loss_tensor_validation(preds, target, self.num_classes, self.ignore_index, self._validation_sink(target))
        preds, target = multiclass_format(preds, target, self.ignore_index, convert_to_labels=False)
        measures, total = _multiclass_hinge_loss_update(preds, target, self.squared, self.multiclass_mode)
        self.measures += measures
        self.total += total


class HingeLoss(_ClassificationTaskWrapper):
    def __new__(  # type: ignore[misc]
        cls: Type["HingeLoss"],
        task: Literal["binary", "multiclass"],
        num_classes: Optional[int] = None,
        squared: bool = False,
        multiclass_mode: Optional[Literal["crammer-singer", "one-vs-all"]] = "crammer-singer",
        ignore_index: Optional[int] = None,
        validate_args: bool = True,
        **kwargs: Any,
    ) -> Metric:
        task = ClassificationTaskNoMultilabel.from_str(task)
        kwargs.update({"ignore_index": ignore_index, "validate_args": validate_args})
        if task == ClassificationTaskNoMultilabel.BINARY:
            return BinaryHingeLoss(squared, **kwargs)
        if not isinstance(num_classes, int):
            raise ValueError(f"`num_classes` is expected to be `int` but `{type(num_classes)} was passed.`")
        return MulticlassHingeLoss(num_classes, squared, multiclass_mode, **kwargs)
