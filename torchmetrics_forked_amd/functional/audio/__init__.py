"""Functional audio metrics (reference ``functional/audio/__init__.py``)."""
from torchmetrics_forked_amd.functional.audio.pesq import perceptual_evaluation_speech_quality
from torchmetrics_forked_amd.functional.audio.pit import permutation_invariant_training, pit_permutate
from torchmetrics_forked_amd.functional.audio.sdr import (
    scale_invariant_signal_distortion_ratio,
    signal_distortion_ratio,
    source_aggregated_signal_distortion_ratio,
)
from torchmetrics_forked_amd.functional.audio.snr import (
    complex_scale_invariant_signal_noise_ratio,
    scale_invariant_signal_noise_ratio,
    signal_noise_ratio,
)
from torchmetrics_forked_amd.functional.audio.srmr import speech_reverberation_modulation_energy_ratio
from torchmetrics_forked_amd.functional.audio.stoi import short_time_objective_intelligibility

__all__ = [
    "permutation_invariant_training",
    "pit_permutate",
    "scale_invariant_signal_distortion_ratio",
    "source_aggregated_signal_distortion_ratio",
    "signal_distortion_ratio",
    "scale_invariant_signal_noise_ratio",
    "signal_noise_ratio",
    "complex_scale_invariant_signal_noise_ratio",
    "perceptual_evaluation_speech_quality",
    "short_time_objective_intelligibility",
    "speech_reverberation_modulation_energy_ratio",
]
