"""Cohen's kappa modules (API parity: reference ``classification/cohen_kappa.py:31-265``).

State = the confusion matrix (``sum``-reduced), filled by the fused confusion-matrix kernels."""
from typing import Any, Optional, Type

from torch import Tensor
from typing_extensions import Literal

from torchmetrics_forked_amd.classification.base import _ClassificationTaskWrapper
from torchmetrics_forked_amd.classification.confusion_matrix import BinaryConfusionMatrix, MulticlassConfusionMatrix
from torchmetrics_forked_amd.functional.classification.cohen_kappa import (
    _binary_cohen_kappa_arg_validation,
    _cohen_kappa_reduce,
    _multiclass_cohen_kappa_arg_validation,
)
from torchmetrics_forked_amd.metric import Metric
from torchmetrics_forked_amd.utilities.enums import ClassificationTaskNoMultilabel
from torchmetrics_forked_amd.utilities.plot import _AX_TYPE, _PLOT_OUT_TYPE


class BinaryCohenKappa(BinaryConfusionMatrix):
    """BinaryCohenKappa (binary task).

    Example:
        >>> import torch
        >>> from torchmetrics_forked_amd.classification import BinaryCohenKappa
        >>> preds = torch.tensor([0.1, 0.8, 0.6, 0.3, 0.9, 0.2])
        >>> target = torch.tensor([0, 1, 0, 0, 1, 1])
        >>> metric = BinaryCohenKappa()
        >>> metric(preds, target)
        tensor(0.3333)
    """
    is_differentiable: bool = False
    higher_is_better: bool = True
    full_state_update: bool = False
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0

    def __init__(
        self,
        threshold: float = 0.5,
        ignore_index: Optional[int] = None,
        weights: Optional[Literal["linear", "quadratic", "none"]] = None,
        validate_args: bool = True,
        **kwargs: Any,
    ) -> None:
        super().__init__(threshold, ignore_index, normalize=None, validate_args=False, **kwargs)
        if validate_args:
            _binary_cohen_kappa_arg_validation(threshold, ignore_index, weights)
        self.weights = weights
        self.validate_args = validate_args

    def compute(self) -> Tensor:
        return _cohen_kappa_reduce(self.confmat, self.weights)

    def plot(self, val: Optional[Tensor] = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:  # type: ignore[override]
        return self._plot(val, ax)


class MulticlassCohenKappa(MulticlassConfusionMatrix):
    """Cohen's kappa for multiclass tasks.

    Example:
        >>> import torch
        >>> from torchmetrics_forked_amd.classification import MulticlassCohenKappa
        >>> MulticlassCohenKappa(num_classes=3)(torch.tensor([2, 1, 0, 1]), torch.tensor([2, 1, 0, 0]))
        tensor(0.6364)
    """
    is_differentiable: bool = False
    higher_is_better: bool = True
    full_state_update: bool = False
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0

    def __init__(
        self,
        num_classes: int,
        ignore_index: Optional[int] = None,
        weights: Optional[Literal["linear", "quadratic", "none"]] = None,
        validate_args: bool = True,
        **kwargs: Any,
    ) -> None:
        super().__init__(num_classes, ignore_index, normalize=None, validate_args=False, **kwargs)
        if validate_args:
            _multiclass_cohen_kappa_arg_validation(num_classes, ignore_index, weights)
        self.weights = weights
        self.validate_args = validate_args

    def compute(self) -> Tensor:
        return _cohen_kappa_reduce(self.confmat, self.weights)

    def plot(self, val: Optional[Tensor] = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:  # type: ignore[override]
        return self._plot(val, ax)


class CohenKappa(_ClassificationTaskWrapper):
    def __new__(  # type: ignore[misc]
        cls: Type["CohenKappa"],
        task: Literal["binary", "multiclass"],
        threshold: float = 0.5,
        num_classes: Optional[int] = None,
        weights: Optional[Literal["linear", "quadratic", "none"]] = None,
        ignore_index: Optional[int] = None,
        validate_args: bool = True,
        **kwargs: Any,
    ) -> Metric:
        task = ClassificationTaskNoMultilabel.from_str(task)
        kwargs.update({"weights": weights, "ignore_index": ignore_index, "validate_args": validate_args})
        if task == ClassificationTaskNoMultilabel.BINARY:
            return BinaryCohenKappa(threshold, **kwargs)
        if not isinstance(num_classes, int):
            raise ValueError(f"`num_classes` is expected to be `int` but `{type(num_classes)} was passed.`")
        return MulticlassCohenKappa(num_classes, **kwargs)
