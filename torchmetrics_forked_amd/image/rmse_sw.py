"""Module-path alias of reference ``src/torchmetrics/image/rmse_sw.py`` (the implementation lives in ``torchmetrics_forked_amd.image``;
this file keeps ``from torchmetrics.image.rmse_sw import ...`` style imports working)."""
from torchmetrics_forked_amd.image import RootMeanSquaredErrorUsingSlidingWindow

__all__ = ['RootMeanSquaredErrorUsingSlidingWindow']
