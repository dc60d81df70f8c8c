"""Precision / Recall modules (API parity: reference classification/precision_recall.py:38-1021).

Each class reuses its ``*StatScores`` parent for state + fused update and only changes ``compute``.
"""
from typing import Any, Optional, Sequence, Type, Union

from torch import Tensor
from typing_extensions import Literal

from torchmetrics_forked_amd.classification.base import _ClassificationTaskWrapper
from torchmetrics_forked_amd.classification.stat_scores import (
    BinaryStatScores,
    MulticlassStatScores,
    MultilabelStatScores,
    _task_factory,
)
from torchmetrics_forked_amd.functional.classification._stat_family import _precision_recall_reduce
from torchmetrics_forked_amd.metric import Metric
from torchmetrics_forked_amd.utilities.plot import _AX_TYPE, _PLOT_OUT_TYPE
from functools import partial


class BinaryPrecision(BinaryStatScores):
    """Precision for binary tasks.

    Example:
        >>> import torch
        >>> from torchmetrics_forked_amd.classification import BinaryPrecision
        >>> preds = torch.tensor([0.1, 0.8, 0.6, 0.3, 0.9, 0.2])
        >>> target = torch.tensor([0, 1, 0, 0, 1, 1])
        >>> metric = BinaryPrecision()
        >>> metric(preds, target)
        tensor(0.6667)
    """

    is_differentiable: bool = False
    higher_is_better: Optional[bool] = True
    full_state_update: bool = False
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0

    def compute(self) -> Tensor:
        tp, fp, tn, fn = self._final_state()
        return partial(_precision_recall_reduce, "precision")(tp, fp, tn, fn, average="binary", multidim_average=self.multidim_average)


class MulticlassPrecision(MulticlassStatScores):
    """Precision for multiclass tasks.

    Example:
        >>> import torch
        >>> from torchmetrics_forked_amd.classification import MulticlassPrecision
        >>> metric = MulticlassPrecision(num_classes=3, average='micro')
        >>> metric(torch.tensor([2, 1, 0, 1]), torch.tensor([2, 1, 0, 0]))
        tensor(0.7500)
    """

    is_differentiable: bool = False
    higher_is_better: Optional[bool] = True
    full_state_update: bool = False
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0
    plot_legend_name: str = "Class"

    def compute(self) -> Tensor:
        tp, fp, tn, fn = self._final_state()
        return partial(_precision_recall_reduce, "precision")(tp, fp, tn, fn, average=self.average, multidim_average=self.multidim_average)


class MultilabelPrecision(MultilabelStatScores):
    """Precision for multilabel tasks.

    Example:
        >>> import torch
        >>> from torchmetrics_forked_amd.classification import MultilabelPrecision
        >>> preds = torch.tensor([[0.2, 0.9, 0.1], [0.7, 0.4, 0.3], [0.6, 0.8, 0.9]])
        >>> target = torch.tensor([[0, 1, 0], [1, 0, 1], [1, 1, 0]])
        >>> metric = MultilabelPrecision(num_labels=3)
        >>> metric(preds, target)
        tensor(0.6667)
    """

    is_differentiable: bool = False
    higher_is_better: Optional[bool] = True
    full_state_update: bool = False
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0
    plot_legend_name: str = "Label"

    def compute(self) -> Tensor:
        tp, fp, tn, fn = self._final_state()
        return partial(_precision_recall_reduce, "precision")(tp, fp, tn, fn, average=self.average, multidim_average=self.multidim_average, multilabel=True)


class Precision(_ClassificationTaskWrapper):
    """Task wrapper: returns Binary/Multiclass/MultilabelPrecision."""

    def __new__(  # type: ignore[misc]
        cls: Type["Precision"],
        task: Literal["binary", "multiclass", "multilabel"],
        threshold: float = 0.5,
        num_classes: Optional[int] = None,
        num_labels: Optional[int] = None,
        average: Optional[Literal["micro", "macro", "weighted", "none"]] = "micro",
        multidim_average: Literal["global", "samplewise"] = "global",
        top_k: Optional[int] = 1,
        ignore_index: Optional[int] = None,
        validate_args: bool = True,
        **kwargs: Any,
    ) -> Metric:
        kwargs.update({"multidim_average": multidim_average, "ignore_index": ignore_index, "validate_args": validate_args})
        return _task_factory(
            task, BinaryPrecision, MulticlassPrecision, MultilabelPrecision,
            (threshold,), (num_classes, top_k, average), (num_labels, threshold, average),
            num_classes, num_labels, top_k, kwargs,
        )


class BinaryRecall(BinaryStatScores):
    """Recall for binary tasks.

    Example:
        >>> import torch
        >>> from torchmetrics_forked_amd.classification import BinaryRecall
        >>> preds = torch.tensor([0.1, 0.8, 0.6, 0.3, 0.9, 0.2])
        >>> target = torch.tensor([0, 1, 0, 0, 1, 1])
        >>> metric = BinaryRecall()
        >>> metric(preds, target)
        tensor(0.6667)
    """

    is_differentiable: bool = False
    higher_is_better: Optional[bool] = True
    full_state_update: bool = False
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0

    def compute(self) -> Tensor:
        tp, fp, tn, fn = self._final_state()
        return partial(_precision_recall_reduce, "recall")(tp, fp, tn, fn, average="binary", multidim_average=self.multidim_average)


class MulticlassRecall(MulticlassStatScores):
    """Recall for multiclass tasks.

    Example:
        >>> import torch
        >>> from torchmetrics_forked_amd.classification import MulticlassRecall
        >>> metric = MulticlassRecall(num_classes=3, average=None)
        >>> metric(torch.tensor([2, 1, 0, 1]), torch.tensor([2, 1, 0, 0]))
        tensor([0.5000, 1.0000, 1.0000])
    """

    is_differentiable: bool = False
    higher_is_better: Optional[bool] = True
    full_state_update: bool = False
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0
    plot_legend_name: str = "Class"

    def compute(self) -> Tensor:
        tp, fp, tn, fn = self._final_state()
        return partial(_precision_recall_reduce, "recall")(tp, fp, tn, fn, average=self.average, multidim_average=self.multidim_average)


class MultilabelRecall(MultilabelStatScores):
    """Recall for multilabel tasks.

    Example:
        >>> import torch
        >>> from torchmetrics_forked_amd.classification import MultilabelRecall
        >>> preds = torch.tensor([[0.2, 0.9, 0.1], [0.7, 0.4, 0.3], [0.6, 0.8, 0.9]])
        >>> target = torch.tensor([[0, 1, 0], [1, 0, 1], [1, 1, 0]])
        >>> metric = MultilabelRecall(num_labels=3)
        >>> metric(preds, target)
        tensor(0.6667)
    """

    is_differentiable: bool = False
    higher_is_better: Optional[bool] = True
    full_state_update: bool = False
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0
    plot_legend_name: str = "Label"

    def compute(self) -> Tensor:
        tp, fp, tn, fn = self._final_state()
        return partial(_precision_recall_reduce, "recall")(tp, fp, tn, fn, average=self.average, multidim_average=self.multidim_average, multilabel=True)


class Recall(_ClassificationTaskWrapper):
    """Task wrapper: returns Binary/Multiclass/MultilabelRecall."""

    def __new__(  # type: ignore[misc]
        cls: Type["Recall"],
        task: Literal["binary", "multiclass", "multilabel"],
        threshold: float = 0.5,
        num_classes: Optional[int] = None,
        num_labels: Optional[int] = None,
        average: Optional[Literal["micro", "macro", "weighted", "none"]] = "micro",
        multidim_average: Literal["global", "samplewise"] = "global",
        top_k: Optional[int] = 1,
        ignore_index: Optional[int] = None,
        validate_args: bool = True,
        **kwargs: Any,
    ) -> Metric:
        kwargs.update({"multidim_average": multidim_average, "ignore_index": ignore_index, "validate_args": validate_args})
        return _task_factory(
            task, BinaryRecall, MulticlassRecall, MultilabelRecall,
            (threshold,), (num_classes, top_k, average), (num_labels, threshold, average),
            num_classes, num_labels, top_k, kwargs,
        )
