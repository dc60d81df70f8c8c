"""Functional text metrics (reference ``functional/text/__init__.py``)."""
from torchmetrics_forked_amd.functional.text.bert import bert_score
from torchmetrics_forked_amd.functional.text.bleu import bleu_score
from torchmetrics_forked_amd.functional.text.cer import char_error_rate
from torchmetrics_forked_amd.functional.text.chrf import chrf_score
from torchmetrics_forked_amd.functional.text.edit import edit_distance
from torchmetrics_forked_amd.functional.text.eed import extended_edit_distance
from torchmetrics_forked_amd.functional.text.infolm import infolm
from torchmetrics_forked_amd.functional.text.mer import match_error_rate
from torchmetrics_forked_amd.functional.text.perplexity import perplexity
from torchmetrics_forked_amd.functional.text.rouge import rouge_score
from torchmetrics_forked_amd.functional.text.sacre_bleu import sacre_bleu_score
from torchmetrics_forked_amd.functional.text.squad import squad
from torchmetrics_forked_amd.functional.text.ter import translation_edit_rate
from torchmetrics_forked_amd.functional.text.wer import word_error_rate
from torchmetrics_forked_amd.functional.text.wil import word_information_lost
from torchmetrics_forked_amd.functional.text.wip import word_information_preserved

__all__ = [
    "bert_score",
    "bleu_score",
    "char_error_rate",
    "chrf_score",
    "edit_distance",
    "extended_edit_distance",
    "infolm",
    "match_error_rate",
    "perplexity",
    "rouge_score",
    "sacre_bleu_score",
    "squad",
    "translation_edit_rate",
    "word_error_rate",
    "word_information_lost",
    "word_information_preserved",
]
