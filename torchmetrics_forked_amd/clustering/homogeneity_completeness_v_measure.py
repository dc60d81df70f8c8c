"""Module-path alias of reference ``src/torchmetrics/clustering/homogeneity_completeness_v_measure.py`` (the implementation lives in ``torchmetrics_forked_amd.clustering``;
this file keeps ``from torchmetrics.clustering.homogeneity_completeness_v_measure import ...`` style imports working)."""
from torchmetrics_forked_amd.clustering import HomogeneityScore, CompletenessScore, VMeasureScore

__all__ = ['HomogeneityScore', 'CompletenessScore', 'VMeasureScore']
