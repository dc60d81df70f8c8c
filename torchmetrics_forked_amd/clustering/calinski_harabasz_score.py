"""Module-path alias of reference ``src/torchmetrics/clustering/calinski_harabasz_score.py`` (the implementation lives in ``torchmetrics_forked_amd.clustering``;
this file keeps ``from torchmetrics.clustering.calinski_harabasz_score import ...`` style imports working)."""
from torchmetrics_forked_amd.clustering import CalinskiHarabaszScore

__all__ = ['CalinskiHarabaszScore']
