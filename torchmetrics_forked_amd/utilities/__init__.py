"""Shared utilities (API parity: reference ``utilities/__init__.py``)."""
from torchmetrics_forked_amd.utilities.checks import check_forward_full_state_property
from torchmetrics_forked_amd.utilities.data import (
    dim_zero_cat,
    dim_zero_max,
    dim_zero_mean,
    dim_zero_min,
    dim_zero_sum,
)
from torchmetrics_forked_amd.utilities.distributed import class_reduce, reduce
from torchmetrics_forked_amd.utilities.prints import rank_zero_debug, rank_zero_info, rank_zero_warn

__all__ = [
    "check_forward_full_state_property",
    "class_reduce",
    "reduce",
    "rank_zero_debug",
    "rank_zero_info",
    "rank_zero_warn",
    "dim_zero_cat",
    "dim_zero_max",
    "dim_zero_mean",
    "dim_zero_min",
    "dim_zero_sum",
]
