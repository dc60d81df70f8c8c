"""Route per-task predictions to per-task metrics (API parity: reference ``wrappers/multitask.py:29-157``)."""
from typing import Any, Dict, Optional, Sequence, Union

from torch import Tensor, nn

from torchmetrics_forked_amd.collections import MetricCollection
from torchmetrics_forked_amd.metric import Metric
from torchmetrics_forked_amd.utilities.plot import _AX_TYPE, _PLOT_OUT_TYPE
from torchmetrics_forked_amd.wrappers.abstract import WrapperMetric


class MultitaskWrapper(WrapperMetric):
    is_differentiable = False

    def __init__(self, task_metrics: Dict[str, Union[Metric, MetricCollection]]) -> None:
        self._check_task_metrics_type(task_metrics)
        super().__init__()
        self.task_metrics = nn.ModuleDict(task_metrics)

    @staticmethod
    def _check_task_metrics_type(task_metrics: Dict[str, Union[Metric, MetricCollection]]) -> None:
        if not isinstance(task_metrics, dict):
            raise TypeError(f"Expected argument `task_metrics` to be a dict. Found task_metrics = {task_metrics}")
        for metric in task_metrics.values():
            if not isinstance(metric, (Metric, MetricCollection)):
                raise TypeError(
                    "Expected each task's metric to be a Metric or a MetricCollection. "
                    f"Found a metric of type {type(metric)}"
                )

    def update(self, task_preds: Dict[str, Tensor], task_targets: Dict[str, Tensor]) -> None:
        if not self.task_metrics.keys() == task_preds.keys() == task_targets.keys():
            raise ValueError(
                "Expected arguments `task_preds` and `task_targets` to have the same keys as the wrapped `task_metrics`"
                f". Found task_preds.keys() = {task_preds.keys()}, task_targets.keys() = {task_targets.keys()} "
                f"and self.task_metrics.keys() = {self.task_metrics.keys()}"
            )
        for name, metric in self.task_metrics.items():
            metric.update(task_preds[name], task_targets[name])

    def compute(self) -> Dict[str, Any]:
        return {name: metric.compute() for name, metric in self.task_metrics.items()}

    def forward(self, task_preds: Dict[str, Tensor], task_targets: Dict[str, Tensor]) -> Dict[str, Any]:
        return {name: metric(task_preds[name], task_targets[name]) for name, metric in self.task_metrics.items()}

    def reset(self) -> None:
        for metric in self.task_metrics.values():
            metric.reset()
        super().reset()

    def plot(self, val: Optional[Union[Dict, Sequence[Dict]]] = None, axes: Optional[Sequence[_AX_TYPE]] = None) -> Sequence[_PLOT_OUT_TYPE]:
        if axes is not None:
            if not isinstance(axes, Sequence):
                raise TypeError(f"Expected argument `axes` to be a Sequence. Found type(axes) = {type(axes)}")
            if len(axes) != len(self.task_metrics):
                raise ValueError(
                    "Expected argument `axes` to be a Sequence of the same length as the number of tasks."
                    f"Found len(axes) = {len(axes)} and {len(self.task_metrics)} tasks"
                )
        val = val if val is not None else self.compute()
        out = []
        for i, (name, metric) in enumerate(self.task_metrics.items()):
            ax = axes[i] if axes is not None else None
            if isinstance(val, dict):
                out.append(metric.plot(val[name], ax=ax))
            elif isinstance(val, Sequence):
                out.append(metric.plot([v[name] for v in val], ax=ax))
            else:
                raise TypeError(
                    f"Expected argument `val` to be None or of type Dict or Sequence[Dict]. Found type(val)= {type(val)}"
                )
        return out
