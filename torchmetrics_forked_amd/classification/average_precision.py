"""Average-precision modules (API parity: reference ``classification/average_precision.py:46-538``).
"""
from typing import Any, List, Optional, Type, Union

from torch import Tensor
from typing_extensions import Literal

from torchmetrics_forked_amd.classification.base import _ClassificationTaskWrapper
from torchmetrics_forked_amd.classification.precision_recall_curve import (
    BinaryPrecisionRecallCurve,
    MulticlassPrecisionRecallCurve,
    MultilabelPrecisionRecallCurve,
    _curve_task_factory,
)
from torchmetrics_forked_amd.functional.classification.precision_recall_curve import (
    _binary_precision_recall_curve_arg_validation,
)
from torchmetrics_forked_amd.functional.classification.auroc import _reduce_auroc
from torchmetrics_forked_amd.functional.classification.average_precision import (
    _multiclass_average_precision_arg_validation,
    _multilabel_average_precision_arg_validation,
    average_precision_compute,
)
from torchmetrics_forked_amd.metric import Metric
from torchmetrics_forked_amd.utilities.plot import _AX_TYPE, _PLOT_OUT_TYPE


class BinaryAveragePrecision(BinaryPrecisionRecallCurve):
    """Average precision for binary tasks.

    Example:
        >>> import torch
        >>> from torchmetrics_forked_amd.classification import BinaryAveragePrecision
        >>> preds = torch.tensor([0.1, 0.8, 0.6, 0.3, 0.9, 0.2])
        >>> target = torch.tensor([0, 1, 0, 0, 1, 1])
        >>> metric = BinaryAveragePrecision()
        >>> metric(preds, target)
        tensor(0.8667)
    """

    is_differentiable: bool = False
    higher_is_better: Optional[bool] = True
    full_state_update: bool = False
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0

    def __init__(
        self,
        thresholds: Optional[Union[int, List[float], Tensor]] = None,
        ignore_index: Optional[int] = None,
        validate_args: bool = True,
        **kwargs: Any,
    ) -> None:
        super().__init__(thresholds=thresholds, ignore_index=ignore_index, validate_args=False, **kwargs)
        if validate_args:
            _binary_precision_recall_curve_arg_validation(thresholds, ignore_index)
        self.validate_args = validate_args

    def compute(self) -> Tensor:
        return average_precision_compute(self._curve_state(), "binary", 1, self.thresholds)

    def plot(self, val: Optional[Union[Tensor, List[Tensor]]] = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:
        return self._plot(val, ax)


class MulticlassAveragePrecision(MulticlassPrecisionRecallCurve):
    """One-vs-rest AveragePrecision for multiclass tasks.

    Example:
        >>> import torch
        >>> from torchmetrics_forked_amd.classification import MulticlassAveragePrecision
        >>> preds = torch.tensor([[0.75, 0.05, 0.20], [0.05, 0.75, 0.20], [0.05, 0.05, 0.90], [0.20, 0.10, 0.70]])
        >>> MulticlassAveragePrecision(num_classes=3)(preds, torch.tensor([0, 1, 2, 2]))
        tensor(1.)
    """

    is_differentiable: bool = False
    higher_is_better: Optional[bool] = True
    full_state_update: bool = False
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0
    plot_legend_name: str = "Class"

    def __init__(
        self,
        num_classes: int,
        average: Optional[Literal["macro", "weighted", "none"]] = "macro",
        thresholds: Optional[Union[int, List[float], Tensor]] = None,
        ignore_index: Optional[int] = None,
        validate_args: bool = True,
        **kwargs: Any,
    ) -> None:
        super().__init__(
            num_classes=num_classes, thresholds=thresholds, average=None, ignore_index=ignore_index, validate_args=False, **kwargs
        )
        if validate_args:
            _multiclass_average_precision_arg_validation(num_classes, average, thresholds, ignore_index)
        self.average = average  # type: ignore[assignment]
        self.validate_args = validate_args

    def compute(self) -> Tensor:
        if self._shard_info is not None:  # class-sharded compute (``sharded_compute=True`` under DDP)
            sc = self._sharded_scores()
            _, ap, pos, _ = sc
            return _reduce_auroc(ap.float(), self.average, pos.float(), summary=sc.summary, col=1)
        return average_precision_compute(self._curve_state(lazy=True), "multiclass", self.num_classes, self.thresholds, self.average)

    def plot(self, val: Optional[Union[Tensor, List[Tensor]]] = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:
        return self._plot(val, ax)


class MultilabelAveragePrecision(MultilabelPrecisionRecallCurve):
    """Per-label AveragePrecision (optionally averaged).

    Example:
        >>> import torch
        >>> from torchmetrics_forked_amd.classification import MultilabelAveragePrecision
        >>> preds = torch.tensor([[0.2, 0.9, 0.1], [0.7, 0.4, 0.3], [0.6, 0.8, 0.9]])
        >>> target = torch.tensor([[0, 1, 0], [1, 0, 1], [1, 1, 0]])
        >>> metric = MultilabelAveragePrecision(num_labels=3, average=None)
        >>> metric(preds, target)
        tensor([1.0000, 1.0000, 0.5000])
    """

    is_differentiable: bool = False
    higher_is_better: Optional[bool] = True
    full_state_update: bool = False
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0
    plot_legend_name: str = "Label"

    def __init__(
        self,
        num_labels: int,
        average: Optional[Literal["micro", "macro", "weighted", "none"]] = "macro",
        thresholds: Optional[Union[int, List[float], Tensor]] = None,
        ignore_index: Optional[int] = None,
        validate_args: bool = True,
        **kwargs: Any,
    ) -> None:
        super().__init__(num_labels=num_labels, thresholds=thresholds, ignore_index=ignore_index, validate_args=False, **kwargs)
        if validate_args:
            _multilabel_average_precision_arg_validation(num_labels, average, thresholds, ignore_index)
        self.average = average
        self.validate_args = validate_args

    def compute(self) -> Tensor:
        if self._shard_info is not None:  # label-sharded compute (``sharded_compute=True`` under DDP)
            sc = self._sharded_scores()
            _, ap, pos, _ = sc
            return _reduce_auroc(ap.float(), self.average, pos.float(), summary=sc.summary, col=1)
        return average_precision_compute(
            self._curve_state(), "multilabel", self.num_labels, self.thresholds, self.average, self.ignore_index
        )

    def plot(self, val: Optional[Union[Tensor, List[Tensor]]] = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:
        return self._plot(val, ax)


class AveragePrecision(_ClassificationTaskWrapper):
    """Task wrapper returning Binary/Multiclass/MultilabelAveragePrecision."""

    def __new__(  # type: ignore[misc]
        cls: Type["AveragePrecision"],
        task: Literal["binary", "multiclass", "multilabel"],
        thresholds: Optional[Union[int, List[float], Tensor]] = None,
        num_classes: Optional[int] = None,
        num_labels: Optional[int] = None,
        average: Optional[Literal["macro", "weighted", "none"]] = "macro",
        ignore_index: Optional[int] = None,
        validate_args: bool = True,
        **kwargs: Any,
    ) -> Metric:
        kwargs.update({"thresholds": thresholds, "ignore_index": ignore_index, "validate_args": validate_args})
        return _curve_task_factory(
            task, BinaryAveragePrecision, MulticlassAveragePrecision, MultilabelAveragePrecision,
            (), (num_classes, average), (num_labels, average), num_classes, num_labels, kwargs,
        )
