"""Task-dispatch base (parity: reference ``classification/base.py:19-32``)."""
from typing import Any

from torchmetrics_forked_amd.metric import Metric


class _ClassificationTaskWrapper(Metric):
    """Factories such as ``Accuracy(task=...)`` return the task-specific metric from ``__new__``."""

    def update(self, *args: Any, **kwargs: Any) -> None:
        raise NotImplementedError(
            f"{self.__class__.__name__} metric does not have a global `update` method. Use the task specific metric."
        )

    def compute(self) -> None:
        raise NotImplementedError(
            f"{self.__class__.__name__} metric does not have a global `compute` method. Use the task specific metric."
        )
