"""ROUGEScore (API parity: reference ``text/rouge.py``): per-sentence scores in ``None``-reduced list states
``{rouge_key}_{fmeasure|precision|recall}``, averaged at compute."""
from typing import Any, Callable, Dict, List, Literal, Optional, Sequence, Tuple, Union

from torch import Tensor

from torchmetrics_forked_amd.functional.text.rouge import (
    _NLTK_AVAILABLE,
    ALLOWED_ACCUMULATE_VALUES,
    ALLOWED_ROUGE_KEYS,
    _rouge_score_compute,
    _rouge_score_update,
)
from torchmetrics_forked_amd.metric import Metric
from torchmetrics_forked_amd.utilities.plot import _AX_TYPE, _PLOT_OUT_TYPE


class ROUGEScore(Metric):
    """ROUGE-N / ROUGE-L / ROUGE-Lsum."""

    is_differentiable: bool = False
    higher_is_better: bool = True
    full_state_update: bool = True
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0

    def __init__(
        self,
        use_stemmer: bool = False,
        normalizer: Optional[Callable[[str], str]] = None,
        tokenizer: Optional[Callable[[str], Sequence[str]]] = None,
        accumulate: Literal["avg", "best"] = "best",
        rouge_keys: Union[str, Tuple[str, ...]] = ("rouge1", "rouge2", "rougeL", "rougeLsum"),
        **kwargs: Any,
    ) -> None:
        super().__init__(**kwargs)
        if use_stemmer and not _NLTK_AVAILABLE:
            raise ModuleNotFoundError("Stemmer requires that `nltk` is installed. Use `pip install nltk`.")
        if not isinstance(rouge_keys, tuple):
            rouge_keys = (rouge_keys,)
        for key in rouge_keys:
            if key not in ALLOWED_ROUGE_KEYS:
                raise ValueError(f"Got unknown rouge key {key}. Expected to be one of {ALLOWED_ROUGE_KEYS}")
        if accumulate not in ALLOWED_ACCUMULATE_VALUES:
            raise ValueError(f"Got unknown accumulate value {accumulate}. Expected to be one of {ALLOWED_ACCUMULATE_VALUES}")
        self.rouge_keys = rouge_keys
        self.rouge_keys_values = [ALLOWED_ROUGE_KEYS[k] for k in rouge_keys]
        if use_stemmer:
            import nltk

            self.stemmer = nltk.stem.porter.PorterStemmer()
        else:
            self.stemmer = None
        self.normalizer = normalizer
        self.tokenizer = tokenizer
        self.accumulate = accumulate
        for key in self.rouge_keys:
            for score in ("fmeasure", "precision", "recall"):
                self.add_state(f"{key}_{score}", [], dist_reduce_fx=None)

    def update(self, preds: Union[str, Sequence[str]], target: Union[str, Sequence[str], Sequence[Sequence[str]]]) -> None:
        if isinstance(target, list) and all(isinstance(t, str) for t in target):
            target = [target] if isinstance(preds, str) else [[t] for t in target]
        if isinstance(preds, str):
            preds = [preds]
        if isinstance(target, str):
            target = [[target]]
        out = _rouge_score_update(
            preds, target, self.rouge_keys_values, stemmer=self.stemmer, normalizer=self.normalizer,
            tokenizer=self.tokenizer, accumulate=self.accumulate, device=self.device,
        )
        for key, metrics in out.items():
            for m in metrics:
                for tp, v in m.items():
                    getattr(self, f"rouge{key}_{tp}").append(v.to(self.device))

    def compute(self) -> Dict[str, Tensor]:
        out: Dict[str, List[Tensor]] = {}
        for key in self.rouge_keys_values:
            for tp in ("fmeasure", "precision", "recall"):
                out[f"rouge{key}_{tp}"] = getattr(self, f"rouge{key}_{tp}")
        return _rouge_score_compute(out)

    def __hash__(self) -> int:
        vals = [self.__class__.__name__]
        for key in self._defaults:
            v = getattr(self, key)
            vals.append(tuple(v) if isinstance(v, list) else v)
        return hash(tuple(vals))

    def plot(self, val: Optional[Union[Tensor, Sequence[Tensor]]] = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:
        return self._plot(val, ax)
