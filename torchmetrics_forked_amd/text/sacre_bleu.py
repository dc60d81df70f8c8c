"""Re-export (reference ``text/sacre_bleu.py``)."""
from torchmetrics_forked_amd.text.bleu import SacreBLEUScore

__all__ = ["SacreBLEUScore"]
