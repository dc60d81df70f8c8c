"""MI355X-native metrics framework (capabilities of TorchMetrics 1.3; gfx950 HIP kernels + RCCL sync)."""
import logging as __logging

from torchmetrics_forked_amd.__about__ import __version__  # noqa: F401

_logger = __logging.getLogger("torchmetrics_forked_amd")
_logger.addHandler(__logging.StreamHandler())
_logger.setLevel(__logging.INFO)

from torchmetrics_forked_amd import functional  # noqa: E402
from torchmetrics_forked_amd import image, models, retrieval, wrappers  # noqa: E402,F401
from torchmetrics_forked_amd.aggregation import (  # noqa: E402
    CatMetric,
    MaxMetric,
    MeanMetric,
    MinMetric,
    RunningMean,
    RunningSum,
    SumMetric,
)
from torchmetrics_forked_amd.classification import *  # noqa: E402,F401,F403
from torchmetrics_forked_amd.collections import MetricCollection  # noqa: E402
from torchmetrics_forked_amd.metric import CompositionalMetric, Metric  # noqa: E402
from torchmetrics_forked_amd.nominal import *  # noqa: E402,F401,F403
from torchmetrics_forked_amd.regression import *  # noqa: E402,F401,F403
from torchmetrics_forked_amd.wrappers import (  # noqa: E402
    BootStrapper,
    ClasswiseWrapper,
    MetricTracker,
    MinMaxMetric,
    MultioutputWrapper,
    MultitaskWrapper,
)
