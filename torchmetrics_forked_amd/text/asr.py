"""ASR error-rate modules: WER, CER, MER, WIL, WIP (API parity: reference ``text/wer.py``, ``cer.py``, ``mer.py``,
``wil.py``, ``wip.py``).  Scalar ``sum`` states; every update is one native batched edit-distance call."""
from typing import Any, List, Optional, Sequence, Union

import torch
from torch import Tensor, tensor

from torchmetrics_forked_amd.functional.text.cer import _cer_compute, _cer_update
from torchmetrics_forked_amd.functional.text.mer import _mer_compute, _mer_update
from torchmetrics_forked_amd.functional.text.wer import _wer_compute, _wer_update
from torchmetrics_forked_amd.functional.text.wil import _word_info_lost_compute, _word_info_lost_update
from torchmetrics_forked_amd.functional.text.wip import _wip_compute, _wip_update
from torchmetrics_forked_amd.metric import Metric
from torchmetrics_forked_amd.utilities.plot import _AX_TYPE, _PLOT_OUT_TYPE


class _ErrorsOverTotal(Metric):
    is_differentiable: bool = False
    higher_is_better: bool = False
    full_state_update: bool = False
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0
    errors: Tensor
    total: Tensor
    _update_fn = staticmethod(_wer_update)
    _compute_fn = staticmethod(_wer_compute)

    def __init__(self, **kwargs: Any) -> None:
        super().__init__(**kwargs)
        self.add_state("errors", tensor(0, dtype=torch.float), dist_reduce_fx="sum")
        self.add_state("total", tensor(0, dtype=torch.float), dist_reduce_fx="sum")

    def update(self, preds: Union[str, List[str]], target: Union[str, List[str]]) -> None:
        errors, total = self._update_fn(preds, target, device=self.device)
        self.errors += errors.to(self.errors)
        self.total += total.to(self.total)

    def compute(self) -> Tensor:
        return self._compute_fn(self.errors, self.total)

    def plot(self, val: Optional[Union[Tensor, Sequence[Tensor]]] = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:
        return self._plot(val, ax)


class WordErrorRate(_ErrorsOverTotal):
    """Word error rate.

    Example:
        >>> from torchmetrics_forked_amd.text import WordErrorRate
        >>> WordErrorRate()(['this is the prediction', 'there is an other sample'], ['this is the reference', 'there is another one'])
        tensor(0.5000)
    """


class CharErrorRate(_ErrorsOverTotal):
    """Character error rate.

    Example:
        >>> from torchmetrics_forked_amd.text import CharErrorRate
        >>> CharErrorRate()(['this is the prediction', 'there is an other sample'], ['this is the reference', 'there is another one'])
        tensor(0.3415)
    """

    _update_fn = staticmethod(_cer_update)
    _compute_fn = staticmethod(_cer_compute)


class MatchErrorRate(_ErrorsOverTotal):
    """Match error rate.

    Example:
        >>> from torchmetrics_forked_amd.text import MatchErrorRate
        >>> MatchErrorRate()(['this is the prediction', 'there is an other sample'], ['this is the reference', 'there is another one'])
        tensor(0.4444)
    """

    _update_fn = staticmethod(_mer_update)
    _compute_fn = staticmethod(_mer_compute)


class _WordInfo(Metric):
    is_differentiable: bool = False
    full_state_update: bool = False
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0
    errors: Tensor
    target_total: Tensor
    preds_total: Tensor
    _update_fn = staticmethod(_word_info_lost_update)
    _compute_fn = staticmethod(_word_info_lost_compute)

    def __init__(self, **kwargs: Any) -> None:
        super().__init__(**kwargs)
        self.add_state("errors", tensor(0.0), dist_reduce_fx="sum")
        self.add_state("target_total", tensor(0.0), dist_reduce_fx="sum")
        self.add_state("preds_total", tensor(0.0), dist_reduce_fx="sum")

    def update(self, preds: Union[str, List[str]], target: Union[str, List[str]]) -> None:
        errors, target_total, preds_total = self._update_fn(preds, target, device=self.device)
        self.errors += errors.to(self.errors)
        self.target_total += target_total.to(self.target_total)
        self.preds_total += preds_total.to(self.preds_total)

    def compute(self) -> Tensor:
        return self._compute_fn(self.errors, self.target_total, self.preds_total)

    def plot(self, val: Optional[Union[Tensor, Sequence[Tensor]]] = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:
        return self._plot(val, ax)


class WordInfoLost(_WordInfo):
    """Word information lost.

    Example:
        >>> from torchmetrics_forked_amd.text import WordInfoLost
        >>> WordInfoLost()(['this is the prediction', 'there is an other sample'], ['this is the reference', 'there is another one'])
        tensor(0.6528)
    """

    higher_is_better: bool = False


class WordInfoPreserved(_WordInfo):
    """Word information preserved (the reference flags ``higher_is_better=False`` too; kept for parity)."""

    higher_is_better: bool = False
    _update_fn = staticmethod(_wip_update)
    _compute_fn = staticmethod(_wip_compute)
