"""Text metrics (reference ``text/__init__.py``)."""
from torchmetrics_forked_amd.text.asr import CharErrorRate, MatchErrorRate, WordErrorRate, WordInfoLost, WordInfoPreserved
from torchmetrics_forked_amd.text.bert import BERTScore
from torchmetrics_forked_amd.text.bleu import BLEUScore, SacreBLEUScore
from torchmetrics_forked_amd.text.chrf import CHRFScore
from torchmetrics_forked_amd.text.edit import EditDistance, ExtendedEditDistance, TranslationEditRate
from torchmetrics_forked_amd.text.infolm import InfoLM
from torchmetrics_forked_amd.text.perplexity import Perplexity
from torchmetrics_forked_amd.text.rouge import ROUGEScore
from torchmetrics_forked_amd.text.squad import SQuAD

__all__ = [
    "BERTScore",
    "BLEUScore",
    "CharErrorRate",
    "CHRFScore",
    "EditDistance",
    "ExtendedEditDistance",
    "InfoLM",
    "MatchErrorRate",
    "Perplexity",
    "ROUGEScore",
    "SacreBLEUScore",
    "SQuAD",
    "TranslationEditRate",
    "WordErrorRate",
    "WordInfoLost",
    "WordInfoPreserved",
]
