"""Relative squared error (API parity: reference ``functional/regression/rse.py:22-84``)."""
from typing import Union

import torch
from torch import Tensor

from torchmetrics_forked_amd.functional.regression.r2 import _r2_score_update


def _relative_squared_error_compute(
    sum_squared_obs: Tensor, sum_obs: Tensor, sum_squared_error: Tensor, num_obs: Union[int, Tensor], squared: bool = True
) -> Tensor:
    epsilon = torch.finfo(sum_squared_error.dtype).eps
    rse = sum_squared_error / torch.clamp(sum_squared_obs - sum_obs * sum_obs / num_obs, min=epsilon)
    if not squared:
        rse = torch.sqrt(rse)
    return torch.mean(rse)


def relative_squared_error(preds: Tensor, target: Tensor, squared: bool = True) -> Tensor:
    sso, so, rss, n = _r2_score_update(preds, target)
    return _relative_squared_error_compute(sso, so, rss, n, squared=squared)
