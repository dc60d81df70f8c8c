"""Deprecated ``functional`` root-import shims for ``text`` (reference ``functional/text/_deprecated.py``)."""
from torchmetrics_forked_amd.functional.text import (
    bleu_score,
    char_error_rate,
    chrf_score,
    extended_edit_distance,
    match_error_rate,
    perplexity,
    rouge_score,
    sacre_bleu_score,
    squad,
    translation_edit_rate,
    word_error_rate,
    word_information_lost,
    word_information_preserved,
    bert_score,
    infolm,
)
from torchmetrics_forked_amd.utilities.deprecation import deprecated_func

_bleu_score = deprecated_func(bleu_score, "text")
_char_error_rate = deprecated_func(char_error_rate, "text")
_chrf_score = deprecated_func(chrf_score, "text")
_extended_edit_distance = deprecated_func(extended_edit_distance, "text")
_match_error_rate = deprecated_func(match_error_rate, "text")
_perplexity = deprecated_func(perplexity, "text")
_rouge_score = deprecated_func(rouge_score, "text")
_sacre_bleu_score = deprecated_func(sacre_bleu_score, "text")
_squad = deprecated_func(squad, "text")
_translation_edit_rate = deprecated_func(translation_edit_rate, "text")
_word_error_rate = deprecated_func(word_error_rate, "text")
_word_information_lost = deprecated_func(word_information_lost, "text")
_word_information_preserved = deprecated_func(word_information_preserved, "text")
_bert_score = deprecated_func(bert_score, "text")
_infolm = deprecated_func(infolm, "text")
