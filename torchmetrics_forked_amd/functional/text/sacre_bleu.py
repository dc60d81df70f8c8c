"""SacreBLEU (API parity: reference ``functional/text/sacre_bleu.py``; tokenisers of the sacrebleu package).

``13a`` / ``zh`` / ``intl`` / ``char`` / ``none`` are implemented here; ``ja-mecab`` / ``ko-mecab`` need their
external analysers and ``flores101`` / ``flores200`` need the sentencepiece model file already present in
``$TMPDIR/torchmetrics-flores`` (nothing is downloaded)."""
import os
import re
import tempfile
from functools import partial
from typing import Any, ClassVar, Dict, Literal, Optional, Sequence, Type, Union

import torch
from torch import Tensor, tensor

from torchmetrics_forked_amd.functional.text.bleu import _bleu_score_compute, _bleu_score_update
from torchmetrics_forked_amd.utilities.imports import package_available

AVAILABLE_TOKENIZERS = ("none", "13a", "zh", "intl", "char", "ja-mecab", "ko-mecab", "flores101", "flores200")
_TokenizersLiteral = Literal["none", "13a", "zh", "intl", "char", "ja-mecab", "ko-mecab", "flores101", "flores200"]

# CJK ranges of sacrebleu's zh tokenizer (string comparison, kept verbatim including its two 5-digit entries)
_UCODE_RANGES = (
    ("\u3400", "\u4db5"), ("\u4e00", "\u9fa5"), ("\u9fa6", "\u9fbb"), ("\uf900", "\ufa2d"),
    ("\ufa30", "\ufa6a"), ("\ufa70", "\ufad9"), ("\u20000", "\u2a6d6"), ("\u2f800", "\u2fa1d"),
    ("\uff00", "\uffef"), ("\u2e80", "\u2eff"), ("\u3000", "\u303f"), ("\u31c0", "\u31ef"),
    ("\u2f00", "\u2fdf"), ("\u2ff0", "\u2fff"), ("\u3100", "\u312f"), ("\u31a0", "\u31bf"),
    ("\ufe10", "\ufe1f"), ("\ufe30", "\ufe4f"), ("\u2600", "\u26ff"), ("\u2700", "\u27bf"),
    ("\u3200", "\u32ff"), ("\u3300", "\u33ff"),
)
_FLORES_LOCAL_DIR = os.path.join(tempfile.gettempdir(), "torchmetrics-flores")
_FLORES_FILES = {"flores101": "sacrebleu_tokenizer_spm.model", "flores200": "flores200sacrebleuspm"}
_REGEX_AVAILABLE = package_available("regex")


class _SacreBLEUTokenizer:
    _REGEX = (
        (re.compile(r"([\{-\~\[-\` -\&\(-\+\:-\@\/])"), r" \1 "),
        (re.compile(r"([^0-9])([\.,])"), r"\1 \2 "),
        (re.compile(r"([\.,])([^0-9])"), r" \1 \2"),
        (re.compile(r"([0-9])(-)"), r"\1 \2 "),
    )
    _TOKENIZE_FN: ClassVar[dict] = {
        "none": "_tokenize_base",
        "13a": "_tokenize_13a",
        "zh": "_tokenize_zh",
        "intl": "_tokenize_international",
        "char": "_tokenize_char",
        "ja-mecab": "_tokenize_ja_mecab",
        "ko-mecab": "_tokenize_ko_mecab",
        "flores101": "_tokenize_flores_101",
        "flores200": "_tokenize_flores_200",
    }
    sentencepiece_processors: ClassVar[Dict[str, Optional[Any]]] = {"flores101": None, "flores200": None}
    _int_regex: ClassVar[Optional[tuple]] = None

    def __init__(self, tokenize: _TokenizersLiteral, lowercase: bool = False) -> None:
        self._check_tokenizers_validity(tokenize)
        self.tokenize_fn = getattr(self, self._TOKENIZE_FN[tokenize])
        self.lowercase = lowercase

    def __call__(self, line: str) -> Sequence[str]:
        return self._lower(self.tokenize_fn(line), self.lowercase).split()

    @classmethod
    def tokenize(cls: Type["_SacreBLEUTokenizer"], line: str, tokenize: _TokenizersLiteral, lowercase: bool = False) -> Sequence[str]:
        cls._check_tokenizers_validity(tokenize)
        return cls._lower(getattr(cls, cls._TOKENIZE_FN[tokenize])(line), lowercase).split()

    @classmethod
    def _tokenize_regex(cls, line: str) -> str:
        for pat, rep in cls._REGEX:
            line = pat.sub(rep, line)
        return " ".join(line.split())

    @staticmethod
    def _is_chinese_char(uchar: str) -> bool:
        return any(start <= uchar <= end for start, end in _UCODE_RANGES)

    @classmethod
    def _tokenize_base(cls, line: str) -> str:
        return line

    @classmethod
    def _tokenize_13a(cls, line: str) -> str:
        line = line.replace("<skipped>", "").replace("-\n", "").replace("\n", " ")
        if "&" in line:
            line = line.replace("&quot;", '"').replace("&amp;", "&").replace("&lt;", "<").replace("&gt;", ">")
        return cls._tokenize_regex(f" {line} ")

    @classmethod
    def _tokenize_zh(cls, line: str) -> str:
        out = "".join(f" {c} " if cls._is_chinese_char(c) else c for c in line.strip())
        return cls._tokenize_regex(out)

    @classmethod
    def _tokenize_international(cls, line: str) -> str:
        if cls._int_regex is None:
            import regex

            cls._int_regex = (
                (regex.compile(r"(\P{N})(\p{P})"), r"\1 \2 "),
                (regex.compile(r"(\p{P})(\P{N})"), r" \1 \2"),
                (regex.compile(r"(\p{S})"), r" \1 "),
            )
        for pat, rep in cls._int_regex:
            line = pat.sub(rep, line)
        return " ".join(line.split())

    @classmethod
    def _tokenize_char(cls, line: str) -> str:
        return " ".join(c for c in line)

    @classmethod
    def _tokenize_ja_mecab(cls, line: str) -> str:
        import ipadic
        import MeCab

        return MeCab.Tagger(ipadic.MECAB_ARGS + " -Owakati").parse(line.strip()).strip()

    @classmethod
    def _tokenize_ko_mecab(cls, line: str) -> str:
        import mecab_ko
        import mecab_ko_dic

        return mecab_ko.Tagger(mecab_ko_dic.MECAB_ARGS + " -Owakati").parse(line.strip()).strip()

    @classmethod
    def _tokenize_flores(cls, line: str, tokenize: Literal["flores101", "flores200"]) -> str:
        import sentencepiece

        if cls.sentencepiece_processors[tokenize] is None:
            path = os.path.join(_FLORES_LOCAL_DIR, _FLORES_FILES[tokenize])
            if not os.path.exists(path):
                raise FileNotFoundError(
                    f"`{tokenize}` tokenization needs the sentencepiece model at {path} (no download is attempted)."
                )
            proc = sentencepiece.SentencePieceProcessor()
            proc.Load(path)
            cls.sentencepiece_processors[tokenize] = proc
        return " ".join(cls.sentencepiece_processors[tokenize].EncodeAsPieces(line))

    @classmethod
    def _tokenize_flores_101(cls, line: str) -> str:
        return cls._tokenize_flores(line, "flores101")

    @classmethod
    def _tokenize_flores_200(cls, line: str) -> str:
        return cls._tokenize_flores(line, "flores200")

    @staticmethod
    def _lower(line: str, lowercase: bool) -> str:
        return line.lower() if lowercase else line

    @classmethod
    def _check_tokenizers_validity(cls, tokenize: _TokenizersLiteral) -> None:
        if tokenize not in cls._TOKENIZE_FN:
            raise ValueError(f"Unsupported tokenizer selected. Please, choose one of {list(cls._TOKENIZE_FN.keys())}")
        if tokenize == "intl" and not _REGEX_AVAILABLE:
            raise ModuleNotFoundError("`'intl'` tokenization requires that `regex` is installed.")
        if tokenize == "ja-mecab" and not (package_available("MeCab") and package_available("ipadic")):
            raise ModuleNotFoundError("`'ja-mecab'` tokenization requires that `MeCab` and `ipadic` are installed.")
        if tokenize == "ko-mecab" and not (package_available("mecab_ko") and package_available("mecab_ko_dic")):
            raise ModuleNotFoundError("`'ko-mecab'` tokenization requires that `mecab_ko` and `mecab_ko_dic` are installed.")
        if "flores" in tokenize and not package_available("sentencepiece"):
            raise ModuleNotFoundError("`'flores101' and 'flores200'` tokenizations require that `sentencepiece` is installed.")


def sacre_bleu_score(
    preds: Sequence[str],
    target: Sequence[Sequence[str]],
    n_gram: int = 4,
    smooth: bool = False,
    tokenize: _TokenizersLiteral = "13a",
    lowercase: bool = False,
    weights: Optional[Sequence[float]] = None,
) -> Tensor:
    """Corpus BLEU with sacrebleu tokenisation."""
    if len(preds) != len(target):
        raise ValueError(f"Corpus has different size {len(preds)} != {len(target)}")
    if weights is not None and len(weights) != n_gram:
        raise ValueError(f"List of weights has different weights than `n_gram`: {len(weights)} != {n_gram}")
    if weights is None:
        weights = [1.0 / n_gram] * n_gram
    numerator = torch.zeros(n_gram)
    denominator = torch.zeros(n_gram)
    tokenize_fn = partial(_SacreBLEUTokenizer.tokenize, tokenize=tokenize, lowercase=lowercase)
    preds_len, target_len = _bleu_score_update(
        preds, target, numerator, denominator, tensor(0.0), tensor(0.0), n_gram, tokenize_fn
    )
    return _bleu_score_compute(preds_len, target_len, numerator, denominator, n_gram, weights, smooth)
