"""Functional multimodal metrics (reference ``functional/multimodal/__init__.py``)."""
from torchmetrics_forked_amd.functional.multimodal.clip_iqa import clip_image_quality_assessment
from torchmetrics_forked_amd.functional.multimodal.clip_score import clip_score

__all__ = ["clip_score", "clip_image_quality_assessment"]
