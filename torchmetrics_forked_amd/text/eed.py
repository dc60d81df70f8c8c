"""Re-export (reference ``text/eed.py``)."""
from torchmetrics_forked_amd.text.edit import ExtendedEditDistance

__all__ = ["ExtendedEditDistance"]
