"""Re-export (reference ``text/wip.py``)."""
from torchmetrics_forked_amd.text.asr import WordInfoPreserved

__all__ = ["WordInfoPreserved"]
