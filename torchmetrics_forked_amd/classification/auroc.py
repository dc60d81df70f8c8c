"""AUROC modules (API parity: reference ``classification/auroc.py:43-541``).

``MulticlassAUROC`` with ``thresholds=None`` on bf16/fp16 scores keeps the exact ``int64 [C, 2, 16384]``
histogram state: the update is one fused HIP pass (softmax-if-needed + code histogram), the cross-rank sync is a
single RCCL all-reduce, and ``compute`` scores all classes in one kernel.
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
from torchmetrics_forked_amd.functional.classification.auroc import (
    _reduce_auroc,
    _warn_degenerate,
    _binary_auroc_arg_validation,
    _multiclass_auroc_arg_validation,
    _multilabel_auroc_arg_validation,
    auroc_compute,
)
from torchmetrics_forked_amd.metric import Metric
from torchmetrics_forked_amd.utilities.plot import _AX_TYPE, _PLOT_OUT_TYPE


class BinaryAUROC(BinaryPrecisionRecallCurve):
    """Area under the ROC curve for binary tasks.

    Example:
        >>> import torch
        >>> from torchmetrics_forked_amd.classification import BinaryAUROC
        >>> metric = BinaryAUROC()
        >>> metric(torch.tensor([0.1, 0.4, 0.35, 0.8]), torch.tensor([0, 0, 1, 1]))
        tensor(0.7500)
    """

    is_differentiable: bool = False
    higher_is_better: Optional[bool] = True
    full_state_update: bool = False
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0

    def __init__(
        self,
        max_fpr: Optional[float] = None,
        thresholds: Optional[Union[int, List[float], Tensor]] = None,
        ignore_index: Optional[int] = None,
        validate_args: bool = True,
        **kwargs: Any,
    ) -> None:
        super().__init__(thresholds=thresholds, ignore_index=ignore_index, validate_args=False, **kwargs)
        if validate_args:
            _binary_auroc_arg_validation(max_fpr, thresholds, ignore_index)
        self.max_fpr = max_fpr
        self.validate_args = validate_args

    def compute(self) -> Tensor:
        return auroc_compute(self._curve_state(), "binary", 1, self.thresholds, max_fpr=self.max_fpr)

    def plot(self, val: Optional[Union[Tensor, List[Tensor]]] = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:
        return self._plot(val, ax)


class MulticlassAUROC(MulticlassPrecisionRecallCurve):
    """One-vs-rest AUROC for multiclass tasks.

    Example:
        >>> import torch
        >>> from torchmetrics_forked_amd.classification import MulticlassAUROC
        >>> preds = torch.tensor([[0.75, 0.05, 0.20], [0.05, 0.75, 0.20], [0.05, 0.05, 0.90], [0.20, 0.10, 0.70]])
        >>> target = torch.tensor([0, 1, 2, 2])
        >>> MulticlassAUROC(num_classes=3)(preds, target)
        tensor(1.)
        >>> MulticlassAUROC(num_classes=3, average=None)(preds, target)
        tensor([1., 1., 1.])
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
            _multiclass_auroc_arg_validation(num_classes, average, thresholds, ignore_index)
        self.average = average  # type: ignore[assignment]
        self.validate_args = validate_args

    def compute(self) -> Tensor:
        if self._shard_info is not None:  # class-sharded compute (``sharded_compute=True`` under DDP)
            sc = self._sharded_scores()
            auc, _, pos, neg = sc
            _warn_degenerate(pos, neg, sc.summary)
            return _reduce_auroc(auc.float(), self.average, pos.float(), summary=sc.summary, col=0)
        return auroc_compute(self._curve_state(lazy=True), "multiclass", self.num_classes, self.thresholds, self.average)

    def plot(self, val: Optional[Union[Tensor, List[Tensor]]] = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:
        return self._plot(val, ax)


class MultilabelAUROC(MultilabelPrecisionRecallCurve):
    """Per-label AUROC (optionally averaged).

    Example:
        >>> import torch
        >>> from torchmetrics_forked_amd.classification import MultilabelAUROC
        >>> preds = torch.tensor([[0.2, 0.9, 0.1], [0.7, 0.4, 0.3], [0.6, 0.8, 0.9]])
        >>> target = torch.tensor([[0, 1, 0], [1, 0, 1], [1, 1, 0]])
        >>> metric = MultilabelAUROC(num_labels=3, average=None)
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
            _multilabel_auroc_arg_validation(num_labels, average, thresholds, ignore_index)
        self.average = average
        self.validate_args = validate_args

    def compute(self) -> Tensor:
        if self._shard_info is not None:  # label-sharded compute (``sharded_compute=True`` under DDP)
            sc = self._sharded_scores()
            auc, _, pos, neg = sc
            _warn_degenerate(pos, neg, sc.summary)
            return _reduce_auroc(auc.float(), self.average, pos.float(), summary=sc.summary, col=0)
        return auroc_compute(
            self._curve_state(), "multilabel", self.num_labels, self.thresholds, self.average, ignore_index=self.ignore_index
        )

    def plot(self, val: Optional[Union[Tensor, List[Tensor]]] = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:
        return self._plot(val, ax)


class AUROC(_ClassificationTaskWrapper):
    """Task wrapper returning Binary/Multiclass/MultilabelAUROC."""

    def __new__(  # type: ignore[misc]
        cls: Type["AUROC"],
        task: Literal["binary", "multiclass", "multilabel"],
        thresholds: Optional[Union[int, List[float], Tensor]] = None,
        num_classes: Optional[int] = None,
        num_labels: Optional[int] = None,
        average: Optional[Literal["macro", "weighted", "none"]] = "macro",
        max_fpr: Optional[float] = None,
        ignore_index: Optional[int] = None,
        validate_args: bool = True,
        **kwargs: Any,
    ) -> Metric:
        kwargs.update({"thresholds": thresholds, "ignore_index": ignore_index, "validate_args": validate_args})
        return _curve_task_factory(
            task, BinaryAUROC, MulticlassAUROC, MultilabelAUROC,
            (max_fpr,), (num_classes, average), (num_labels, average), num_classes, num_labels, kwargs,
        )
