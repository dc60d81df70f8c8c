"""Shared word/char error statistics for WER / CER / MER / WIL / WIP (reference ``functional/text/wer.py``,
``cer.py``, ``mer.py``, ``wil.py``, ``wip.py``): one native batched edit-distance call per update."""
from typing import List, Optional, Sequence, Tuple, Union

import torch
from torch import Tensor

from torchmetrics_forked_amd.functional.text.helper import _levenshtein_many


def _as_list(x: Union[str, Sequence[str]]) -> List[str]:
    return [x] if isinstance(x, str) else list(x)


def _asr_stats(
    preds: Union[str, Sequence[str]], target: Union[str, Sequence[str]], chars: bool = False, device: Optional[torch.device] = None
) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    """Returns fp32 ``(errors, target_len, pred_len, max_len)`` summed over the pairs (``errors`` on ``device`` when
    the batch was scored on the GPU)."""
    p, t = _as_list(preds), _as_list(target)
    n = min(len(p), len(t))
    p_tok = [list(s) if chars else s.split() for s in p[:n]]
    t_tok = [list(s) if chars else s.split() for s in t[:n]]
    errors = _levenshtein_many(p_tok, t_tok, device).sum().float() if n else torch.tensor(0.0)
    tl = float(sum(len(x) for x in t_tok))
    pl = float(sum(len(x) for x in p_tok))
    ml = float(sum(max(len(a), len(b)) for a, b in zip(p_tok, t_tok)))
    return errors, torch.tensor(tl), torch.tensor(pl), torch.tensor(ml)
