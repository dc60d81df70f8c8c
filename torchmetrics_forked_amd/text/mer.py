"""Re-export (reference ``text/mer.py``)."""
from torchmetrics_forked_amd.text.asr import MatchErrorRate

__all__ = ["MatchErrorRate"]
