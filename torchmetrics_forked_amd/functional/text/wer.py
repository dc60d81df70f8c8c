"""Word error rate (API parity: reference ``functional/text/wer.py``)."""
from typing import List, Optional, Tuple, Union

import torch
from torch import Tensor

from torchmetrics_forked_amd.functional.text._asr import _asr_stats


def _wer_update(
    preds: Union[str, List[str]], target: Union[str, List[str]], device: Optional[torch.device] = None
) -> Tuple[Tensor, Tensor]:
    errors, tl, _, _ = _asr_stats(preds, target, device=device)
    return errors, tl


def _wer_compute(errors: Tensor, total: Tensor) -> Tensor:
    return errors / total


def word_error_rate(preds: Union[str, List[str]], target: Union[str, List[str]]) -> Tensor:
    """Word-level edit operations divided by the number of reference words."""
    errors, total = _wer_update(preds, target)
    return _wer_compute(errors, total)
