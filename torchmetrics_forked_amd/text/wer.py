"""Re-export (reference ``text/wer.py``)."""
from torchmetrics_forked_amd.text.asr import WordErrorRate

__all__ = ["WordErrorRate"]
