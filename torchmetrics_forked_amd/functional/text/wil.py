"""Word information lost (API parity: reference ``functional/text/wil.py``)."""
from typing import List, Optional, Tuple, Union

import torch
from torch import Tensor

from torchmetrics_forked_amd.functional.text._asr import _asr_stats


def _word_info_lost_update(
    preds: Union[str, List[str]], target: Union[str, List[str]], device: Optional[torch.device] = None
) -> Tuple[Tensor, Tensor, Tensor]:
    errors, tl, pl, ml = _asr_stats(preds, target, device=device)
    return errors - ml, tl, pl  # negated hit count (reference convention)


def _word_info_lost_compute(errors: Tensor, target_total: Tensor, preds_total: Tensor) -> Tensor:
    return 1 - ((errors / target_total) * (errors / preds_total))


def word_information_lost(preds: Union[str, List[str]], target: Union[str, List[str]]) -> Tensor:
    """1 - (H / N_target) * (H / N_pred) with H the number of hits."""
    return _word_info_lost_compute(*_word_info_lost_update(preds, target))
