"""BLEUScore / SacreBLEUScore (API parity: reference ``text/bleu.py``, ``text/sacre_bleu.py``)."""
from typing import Any, Optional, Sequence, Union

import torch
from torch import Tensor, tensor

from torchmetrics_forked_amd.functional.text.bleu import _bleu_score_compute, _bleu_score_update, _tokenize_fn
from torchmetrics_forked_amd.functional.text.sacre_bleu import _SacreBLEUTokenizer, _TokenizersLiteral
from torchmetrics_forked_amd.metric import Metric
from torchmetrics_forked_amd.utilities.plot import _AX_TYPE, _PLOT_OUT_TYPE


class BLEUScore(Metric):
    """Corpus BLEU (``sum`` states: lengths and clipped / total n-gram counts).

    Example:
        >>> from torchmetrics_forked_amd.text import BLEUScore
        >>> BLEUScore()(['the squirrel is eating the nut'], [['a squirrel is eating a nut', 'the squirrel is eating a tasty nut']])
        tensor(0.5373)
    """

    is_differentiable: bool = False
    higher_is_better: bool = True
    full_state_update: bool = True
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0
    preds_len: Tensor
    target_len: Tensor
    numerator: Tensor
    denominator: Tensor

    def __init__(self, n_gram: int = 4, smooth: bool = False, weights: Optional[Sequence[float]] = None, **kwargs: Any) -> None:
        super().__init__(**kwargs)
        self.n_gram = n_gram
        self.smooth = smooth
        if weights is not None and len(weights) != n_gram:
            raise ValueError(f"List of weights has different weights than `n_gram`: {len(weights)} != {n_gram}")
        self.weights = weights if weights is not None else [1.0 / n_gram] * n_gram
        self.add_state("preds_len", tensor(0.0), dist_reduce_fx="sum")
        self.add_state("target_len", tensor(0.0), dist_reduce_fx="sum")
        self.add_state("numerator", torch.zeros(self.n_gram), dist_reduce_fx="sum")
        self.add_state("denominator", torch.zeros(self.n_gram), dist_reduce_fx="sum")

    def _tokenizer(self) -> Any:
        return _tokenize_fn

    def update(self, preds: Sequence[str], target: Sequence[Sequence[str]]) -> None:
        self.preds_len, self.target_len = _bleu_score_update(
            preds, target, self.numerator, self.denominator, self.preds_len, self.target_len, self.n_gram, self._tokenizer()
        )

    def compute(self) -> Tensor:
        return _bleu_score_compute(self.preds_len, self.target_len, self.numerator, self.denominator, self.n_gram, self.weights, self.smooth)

    def plot(self, val: Optional[Union[Tensor, Sequence[Tensor]]] = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:
        return self._plot(val, ax)


class SacreBLEUScore(BLEUScore):
    """BLEU with sacrebleu tokenisation.

    Example:
        >>> from torchmetrics_forked_amd.text import SacreBLEUScore
        >>> SacreBLEUScore()(['the squirrel is eating the nut'], [['a squirrel is eating a nut', 'the squirrel is eating a tasty nut']])
        tensor(0.5373)
    """

    def __init__(
        self,
        n_gram: int = 4,
        smooth: bool = False,
        tokenize: _TokenizersLiteral = "13a",
        lowercase: bool = False,
        weights: Optional[Sequence[float]] = None,
        **kwargs: Any,
    ) -> None:
        super().__init__(n_gram=n_gram, smooth=smooth, weights=weights, **kwargs)
        self.tokenizer = _SacreBLEUTokenizer(tokenize, lowercase)

    def _tokenizer(self) -> Any:
        return self.tokenizer
