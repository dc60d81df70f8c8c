"""Curve engine: the state representations behind PR-curve / ROC / AUROC / AP and the fixed-point metrics.

The reference keeps every score in a ``cat`` list and, at compute time, runs one full ``argsort`` *per class*
in a Python loop with several host syncs each (``precision_recall_curve.py:558-563``, ``roc.py:182-187``;
SURVEY §3.5).  Three state kinds are used here instead:

``hist``    exact histogram ``int64 [C, 2, 16384]`` of (class, label, score-code) for bf16/fp16 scores
            (``csrc/classification.hip: curve_hist_update``).  Fixed size -> all-reduced by RCCL instead of
            all-gathered; AUROC / AP for *all* classes come out of one kernel (``curve_hist_reduce``) with no
            per-class loop.  Exact: code order == value order and every distinct score keeps its own bin.
``samples`` ``(preds [N, C], labels [N, C], valid [N, C])`` for fp32/fp64 scores: all classes are sorted at once
            (one segmented sort), tie groups are found with one vectorised pass; no per-class loop for AUROC/AP.
``binned``  the reference's multi-threshold confusion matrix ``[T, C, 2, 2]`` (``binned_curve_update``).

Curve *points* (distinct thresholds with cumulative tps/fps) are produced per class only when a caller asks
for the curves themselves (PR-curve / ROC outputs are ragged lists by API).
"""
from typing import List, Optional, Tuple, Union

import torch
from torch import Tensor

from torchmetrics_forked_amd import ops
from torchmetrics_forked_amd.ops import classification as cls_ops

N_CODES = cls_ops.N_CODES
HIST_DTYPES = (torch.bfloat16, torch.float16)


def codes_to_values(dtype: torch.dtype, device: torch.device) -> Tensor:
    """Value of every code ``0..N_CODES-1`` in ``dtype`` (codes above 1.0 decode to garbage but are never populated)."""
    codes = torch.arange(N_CODES, dtype=torch.int32, device=device)
    return codes.to(torch.int16).view(dtype)


# ---------------------------------------------------------------------------------------------------------
# reductions (AUROC / AP for all classes at once)
# ---------------------------------------------------------------------------------------------------------
def hist_scores(hist: Tensor, code_range: Optional[Tensor] = None) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    """(auroc, ap, n_pos, n_neg) per class from an exact histogram ``[C, 2, K]`` (float64); bins outside
    ``code_range`` ([lo, hi], when given) are known to be empty and are not read."""
    out = cls_ops.curve_hist_reduce(hist, code_range)
    return out[:, 0], out[:, 1], out[:, 2], out[:, 3]


def samples_scores(preds: Tensor, labels: Tensor, valid: Optional[Tensor] = None) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    """(auroc, ap, n_pos, n_neg) per column of ``preds [N, C]`` with binary ``labels [N, C]``.

    ``valid`` masks out ignored entries.  Implemented as: one column-wise sort, tie-group ends via a shifted
    compare, previous-group-end via ``cummax``, then trapezoid / step sums — all vectorised.
    """
    if preds.ndim == 1:
        preds, labels = preds.unsqueeze(1), labels.unsqueeze(1)
        valid = valid.unsqueeze(1) if valid is not None else None
    n, C = preds.shape
    p = preds.float() if preds.dtype in HIST_DTYPES else preds
    lab = labels.to(torch.float64)
    if valid is not None:
        # invalid entries get -inf score and weight 0 (they sort last and never form a group with valid data)
        p = torch.where(valid, p, torch.full_like(p, -float("inf")))
        w = valid.to(torch.float64)
    else:
        w = torch.ones_like(lab)
    if n == 0:
        z = torch.zeros(C, dtype=torch.float64, device=preds.device)
        return z, torch.full_like(z, float("nan")), z, z
    sp, order = torch.sort(p, dim=0, descending=True, stable=True)
    sl = torch.gather(lab, 0, order)
    sw = torch.gather(w, 0, order)
    tps = torch.cumsum(sl * sw, 0)
    fps = torch.cumsum((1 - sl) * sw, 0)
    end = torch.ones_like(sp, dtype=torch.bool)
    end[:-1] = sp[1:] != sp[:-1]
    idx = torch.arange(n, device=p.device).unsqueeze(1).expand(n, C)
    marked = torch.where(end, idx, torch.full_like(idx, -1))
    prev = torch.cummax(marked, 0).values
    prev_end = torch.full_like(prev, -1)
    prev_end[1:] = prev[:-1]
    has_prev = prev_end >= 0
    pe = prev_end.clamp_min(0)
    tps_prev = torch.where(has_prev, torch.gather(tps, 0, pe), torch.zeros_like(tps))
    fps_prev = torch.where(has_prev, torch.gather(fps, 0, pe), torch.zeros_like(fps))
    P, N = tps[-1], fps[-1]
    endf = end.to(torch.float64)
    area = ((fps - fps_prev) * (tps + tps_prev) * endf).sum(0)
    auroc = torch.where((P > 0) & (N > 0), area / (2 * P * N).clamp_min(1e-300), torch.zeros_like(P))
    prec = torch.where(tps + fps > 0, tps / (tps + fps).clamp_min(1e-300), torch.zeros_like(tps))
    ap = torch.where(P > 0, ((tps - tps_prev) * prec * endf).sum(0) / P.clamp_min(1e-300), torch.full_like(P, float("nan")))
    return auroc, ap, P, N


class ColumnChunks:
    """Samples of a multiclass fp32 curve state kept as the class-major ``[C, n_k]`` buffers the GPU update wrote
    (one per ``update``): ``anchored_scores`` streams them in place; everything else calls ``materialize()``."""

    def __init__(self, cols: List[Tensor]) -> None:
        self.cols = cols

    def materialize(self) -> Tensor:
        return torch.cat([c.t() for c in self.cols])


def anchored_scores(
    preds: Union[Tensor, ColumnChunks], target: Tensor, task: str, num: int, ignore_index: Optional[int]
) -> Optional[Tensor]:
    """(auroc, ap, P, N) ``[C, 4]`` from fp32 samples on the GPU through the positive-anchored kernels
    (csrc/curve_anchor.hip: one streaming pass over the class-major scores, only the positives are sorted), or
    ``None`` when the inputs do not qualify: fp64 scores (kept exact in fp64), CPU tensors, multilabel with an
    ``ignore_index``, or a class with more than ``ANCHOR_MAX_POS`` positives (the sort-based path handles those)."""
    if isinstance(preds, ColumnChunks):
        cols = preds.cols
        sample = cols[0]
    else:
        cols, sample = None, preds
    if not (sample.is_cuda and sample.dtype == torch.float32 and ops.use_native(sample)) or target.numel() == 0:
        return None
    if task == "multilabel" and ignore_index is not None:
        return None
    if task == "multiclass":
        C = num
        t = target.reshape(-1).long()
        counts = torch.bincount(t, minlength=C)[:C]
        pos_rows = torch.sort(t, stable=True)[1]
    else:
        p2 = preds.reshape(-1, 1) if task == "binary" else preds
        lab = (target.reshape(p2.shape) == 1).t()
        C = p2.shape[1]
        cls_idx, pos_rows = lab.nonzero(as_tuple=True)
        counts = torch.bincount(cls_idx, minlength=C)
        preds = p2
    max_pos = int(counts.max()) if counts.numel() else 0
    if max_pos > cls_ops.ANCHOR_MAX_POS:
        return None
    pos_off = torch.zeros(C + 1, dtype=torch.long, device=sample.device)
    pos_off[1:] = counts.cumsum(0)
    if cols is None:
        cols = [preds.t().contiguous()]
    return cls_ops.anchored_scores(cols, pos_off, pos_rows, max_pos)


# ---------------------------------------------------------------------------------------------------------
# curve points (fps, tps, thresholds) per class — the `_binary_clf_curve` contract
# ---------------------------------------------------------------------------------------------------------
def hist_curve_points(hist: Tensor, dtype: torch.dtype) -> List[Tuple[Tensor, Tensor, Tensor]]:
    """Per class: (fps, tps, thresholds) at every distinct score, thresholds descending (float32 counts)."""
    C = hist.shape[0]
    neg = hist[:, 0].flip(-1)
    pos = hist[:, 1].flip(-1)
    nz = (neg + pos) > 0
    tps = pos.cumsum(-1).to(torch.float32)
    fps = neg.cumsum(-1).to(torch.float32)
    values = codes_to_values(dtype, hist.device).flip(0).unsqueeze(0).expand(C, -1)
    counts = nz.sum(-1).tolist()
    t_sel, f_sel, v_sel = tps[nz], fps[nz], values[nz]
    out = []
    for a, b, c in zip(torch.split(f_sel, counts), torch.split(t_sel, counts), torch.split(v_sel, counts)):
        out.append((a, b, c))
    return out


def samples_curve_points(preds: Tensor, labels: Tensor) -> Tuple[Tensor, Tensor, Tensor]:
    """(fps, tps, thresholds) for a single 1-D problem (reference ``_binary_clf_curve`` semantics)."""
    with torch.no_grad():
        order = torch.argsort(preds, descending=True)
        sp = preds[order]
        sl = labels[order].to(torch.long)
        distinct = torch.where(sp[1:] - sp[:-1])[0]
        thr_idx = torch.nn.functional.pad(distinct, [0, 1], value=sl.size(0) - 1)
        tps = torch.cumsum(sl * 1.0, dim=0)[thr_idx]
        fps = 1 + thr_idx - tps
        return fps, tps, sp[thr_idx]


def samples_curve_points_columns(preds: Tensor, labels: Tensor) -> List[Tuple[Tensor, Tensor, Tensor]]:
    """(fps, tps, thresholds) for every column of ``preds [N, C]`` against binary ``labels [N, C]``, from ONE batched
    sort of the class-major scores (the reference runs one argsort per class in a Python loop,
    ``precision_recall_curve.py:558-563``).  Ties are merged into one point, so the sort order among equal scores
    does not matter; one host read sizes the per-class outputs."""
    with torch.no_grad():
        cols = preds.t().contiguous()
        sv, order = torch.sort(cols, dim=1, descending=True)
        sl = torch.gather(labels.t().to(torch.float32), 1, order)
        tps = torch.cumsum(sl, dim=1)
        n = cols.shape[1]
        idx = torch.arange(n, device=cols.device, dtype=torch.float32).expand_as(tps)
        fps = idx + 1 - tps
        last = torch.ones_like(sv, dtype=torch.bool)
        last[:, :-1] = sv[:, 1:] != sv[:, :-1]
        counts = last.sum(1).tolist()
        f_sel, t_sel, v_sel = fps[last], tps[last], sv[last]
        return list(zip(torch.split(f_sel, counts), torch.split(t_sel, counts), torch.split(v_sel, counts)))

