"""Metric wrappers (API parity: reference ``wrappers/__init__.py``)."""
from torchmetrics_forked_amd.wrappers.abstract import WrapperMetric
from torchmetrics_forked_amd.wrappers.bootstrapping import BootStrapper
from torchmetrics_forked_amd.wrappers.classwise import ClasswiseWrapper
from torchmetrics_forked_amd.wrappers.minmax import MinMaxMetric
from torchmetrics_forked_amd.wrappers.multioutput import MultioutputWrapper
from torchmetrics_forked_amd.wrappers.multitask import MultitaskWrapper
from torchmetrics_forked_amd.wrappers.running import Running
from torchmetrics_forked_amd.wrappers.tracker import MetricTracker

__all__ = [
    "BootStrapper", "ClasswiseWrapper", "MetricTracker", "MinMaxMetric", "MultioutputWrapper", "MultitaskWrapper",
    "Running", "WrapperMetric",
]
