"""Per-class output to dict (API parity: reference ``wrappers/classwise.py:27-168``)."""
from typing import Any, Dict, List, Optional, Sequence, Union

from torch import Tensor

from torchmetrics_forked_amd.metric import Metric
from torchmetrics_forked_amd.utilities.plot import _AX_TYPE, _PLOT_OUT_TYPE
from torchmetrics_forked_amd.wrappers.abstract import WrapperMetric


class ClasswiseWrapper(WrapperMetric):
    """Splits a per-class metric output into a dict.

    Example:
        >>> import torch
        >>> from torchmetrics_forked_amd.wrappers import ClasswiseWrapper
        >>> from torchmetrics_forked_amd.classification import MulticlassAccuracy
        >>> metric = ClasswiseWrapper(MulticlassAccuracy(num_classes=3, average=None), labels=['cat', 'dog', 'fish'])
        >>> metric(torch.tensor([2, 1, 0, 1]), torch.tensor([2, 1, 0, 0]))
        {'multiclassaccuracy_cat': tensor(0.5000), 'multiclassaccuracy_dog': tensor(1.), 'multiclassaccuracy_fish': tensor(1.)}
    """
    def __init__(
        self, metric: Metric, labels: Optional[List[str]] = None, prefix: Optional[str] = None, postfix: Optional[str] = None
    ) -> None:
        super().__init__()
        if not isinstance(metric, Metric):
            raise ValueError(f"Expected argument `metric` to be an instance of `torchmetrics.Metric` but got {metric}")
        self.metric = metric
        if labels is not None and not (isinstance(labels, list) and all(isinstance(lab, str) for lab in labels)):
            raise ValueError(f"Expected argument `labels` to either be `None` or a list of strings but got {labels}")
        self.labels = labels
        if prefix is not None and not isinstance(prefix, str):
            raise ValueError(f"Expected argument `prefix` to either be `None` or a string but got {prefix}")
        self._prefix = prefix
        if postfix is not None and not isinstance(postfix, str):
            raise ValueError(f"Expected argument `postfix` to either be `None` or a string but got {postfix}")
        self._postfix = postfix
        self._update_count = 1

    def _convert(self, x: Tensor) -> Dict[str, Any]:
        if not self._prefix and not self._postfix:
            prefix, postfix = f"{self.metric.__class__.__name__.lower()}_", ""
        else:
            prefix, postfix = self._prefix or "", self._postfix or ""
        names = range(len(x)) if self.labels is None else self.labels
        return {f"{prefix}{n}{postfix}": v for n, v in zip(names, x)}

    def forward(self, *args: Any, **kwargs: Any) -> Any:
        return self._convert(self.metric(*args, **kwargs))

    def update(self, *args: Any, **kwargs: Any) -> None:
        self.metric.update(*args, **kwargs)

    def compute(self) -> Dict[str, Tensor]:
        return self._convert(self.metric.compute())

    def reset(self) -> None:
        self.metric.reset()

    def plot(self, val: Optional[Union[Tensor, Sequence[Tensor]]] = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:
        return self._plot(val, ax)
