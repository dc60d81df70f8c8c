"""Deprecated ``functional`` root-import shims for ``image`` (reference ``functional/image/_deprecated.py``)."""
from torchmetrics_forked_amd.functional.image import (
    error_relative_global_dimensionless_synthesis,
    image_gradients,
    multiscale_structural_similarity_index_measure,
    peak_signal_noise_ratio,
    relative_average_spectral_error,
    root_mean_squared_error_using_sliding_window,
    spectral_angle_mapper,
    spectral_distortion_index,
    structural_similarity_index_measure,
    total_variation,
    universal_image_quality_index,
)
from torchmetrics_forked_amd.utilities.deprecation import deprecated_func

_error_relative_global_dimensionless_synthesis = deprecated_func(error_relative_global_dimensionless_synthesis, "image")
_image_gradients = deprecated_func(image_gradients, "image")
_multiscale_structural_similarity_index_measure = deprecated_func(multiscale_structural_similarity_index_measure, "image")
_peak_signal_noise_ratio = deprecated_func(peak_signal_noise_ratio, "image")
_relative_average_spectral_error = deprecated_func(relative_average_spectral_error, "image")
_root_mean_squared_error_using_sliding_window = deprecated_func(root_mean_squared_error_using_sliding_window, "image")
_spectral_angle_mapper = deprecated_func(spectral_angle_mapper, "image")
_spectral_distortion_index = deprecated_func(spectral_distortion_index, "image")
_structural_similarity_index_measure = deprecated_func(structural_similarity_index_measure, "image")
_total_variation = deprecated_func(total_variation, "image")
_universal_image_quality_index = deprecated_func(universal_image_quality_index, "image")
