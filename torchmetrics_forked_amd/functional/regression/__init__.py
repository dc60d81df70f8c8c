"""Functional regression metrics (API parity: reference ``functional/regression/__init__.py``).

Sum-state metrics (MSE, MAE, MAPE, SMAPE, WMAPE, MSLE, log-cosh, Minkowski, R2, RSE, explained variance,
Tweedie, Pearson/Concordance moments) read their batch statistics from ONE fused HIP map-reduce pass on the GPU
(``csrc/regression.hip``); rank metrics (Spearman, Kendall) are sort-based and loop-free.
"""
from torchmetrics_forked_amd.functional.regression.concordance import concordance_corrcoef
from torchmetrics_forked_amd.functional.regression.cosine_similarity import cosine_similarity
from torchmetrics_forked_amd.functional.regression.explained_variance import explained_variance
from torchmetrics_forked_amd.functional.regression.kendall import kendall_rank_corrcoef
from torchmetrics_forked_amd.functional.regression.kl_divergence import kl_divergence
from torchmetrics_forked_amd.functional.regression.log_cosh import log_cosh_error
from torchmetrics_forked_amd.functional.regression.log_mse import mean_squared_log_error
from torchmetrics_forked_amd.functional.regression.mae import mean_absolute_error
from torchmetrics_forked_amd.functional.regression.mape import mean_absolute_percentage_error
from torchmetrics_forked_amd.functional.regression.minkowski import minkowski_distance
from torchmetrics_forked_amd.functional.regression.mse import mean_squared_error
from torchmetrics_forked_amd.functional.regression.pearson import pearson_corrcoef
from torchmetrics_forked_amd.functional.regression.r2 import r2_score
from torchmetrics_forked_amd.functional.regression.rse import relative_squared_error
from torchmetrics_forked_amd.functional.regression.spearman import spearman_corrcoef
from torchmetrics_forked_amd.functional.regression.symmetric_mape import symmetric_mean_absolute_percentage_error
from torchmetrics_forked_amd.functional.regression.tweedie_deviance import tweedie_deviance_score
from torchmetrics_forked_amd.functional.regression.wmape import weighted_mean_absolute_percentage_error

__all__ = [
    "concordance_corrcoef", "cosine_similarity", "explained_variance", "kendall_rank_corrcoef", "kl_divergence",
    "log_cosh_error", "mean_squared_log_error", "mean_absolute_error", "mean_squared_error", "pearson_corrcoef",
    "mean_absolute_percentage_error", "minkowski_distance", "r2_score", "relative_squared_error", "spearman_corrcoef",
    "symmetric_mean_absolute_percentage_error", "tweedie_deviance_score", "weighted_mean_absolute_percentage_error",
]
