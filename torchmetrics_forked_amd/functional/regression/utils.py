"""Module-path alias of reference ``src/torchmetrics/functional/regression/utils.py``."""
from torchmetrics_forked_amd.functional.regression._common import _check_data_shape_to_num_outputs

__all__ = ["_check_data_shape_to_num_outputs"]
