"""Module-path alias of reference ``src/torchmetrics/image/mifid.py`` (the implementation lives in ``torchmetrics_forked_amd.image``;
this file keeps ``from torchmetrics.image.mifid import ...`` style imports working)."""
from torchmetrics_forked_amd.image import MemorizationInformedFrechetInceptionDistance

__all__ = ['MemorizationInformedFrechetInceptionDistance']
