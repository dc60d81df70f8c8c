"""Multimodal metrics (reference ``multimodal/__init__.py``)."""
from torchmetrics_forked_amd.multimodal.clip_iqa import CLIPImageQualityAssessment
from torchmetrics_forked_amd.multimodal.clip_score import CLIPScore

__all__ = ["CLIPScore", "CLIPImageQualityAssessment"]
