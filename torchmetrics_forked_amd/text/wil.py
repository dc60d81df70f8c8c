"""Re-export (reference ``text/wil.py``)."""
from torchmetrics_forked_amd.text.asr import WordInfoLost

__all__ = ["WordInfoLost"]
