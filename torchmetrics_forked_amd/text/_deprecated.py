"""Deprecated root-import shims for ``text`` (reference ``text/_deprecated.py``)."""
from torchmetrics_forked_amd.text import (
    BLEUScore,
    CharErrorRate,
    CHRFScore,
    ExtendedEditDistance,
    MatchErrorRate,
    Perplexity,
    SacreBLEUScore,
    SQuAD,
    TranslationEditRate,
    WordErrorRate,
    WordInfoLost,
    WordInfoPreserved,
)
from torchmetrics_forked_amd.utilities.deprecation import deprecated_class

_BLEUScore = deprecated_class(BLEUScore, "text")
_CharErrorRate = deprecated_class(CharErrorRate, "text")
_CHRFScore = deprecated_class(CHRFScore, "text")
_ExtendedEditDistance = deprecated_class(ExtendedEditDistance, "text")
_MatchErrorRate = deprecated_class(MatchErrorRate, "text")
_Perplexity = deprecated_class(Perplexity, "text")
_SacreBLEUScore = deprecated_class(SacreBLEUScore, "text")
_SQuAD = deprecated_class(SQuAD, "text")
_TranslationEditRate = deprecated_class(TranslationEditRate, "text")
_WordErrorRate = deprecated_class(WordErrorRate, "text")
_WordInfoLost = deprecated_class(WordInfoLost, "text")
_WordInfoPreserved = deprecated_class(WordInfoPreserved, "text")
