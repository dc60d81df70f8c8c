"""Re-export (reference ``text/cer.py``)."""
from torchmetrics_forked_amd.text.asr import CharErrorRate

__all__ = ["CharErrorRate"]
