"""Re-export (reference ``text/ter.py``)."""
from torchmetrics_forked_amd.text.edit import TranslationEditRate

__all__ = ["TranslationEditRate"]
