"""Curve engine: the state representations behind PR-curve / ROC / AUROC / AP and the fixed-point metrics.

The reference keeps every score in a ``cat`` list and, at compute time, runs one full ``argsort`` *per class*
in a Python loop with several host syncs each (``precision_recall_curve.py:558-563``, ``roc.py:182-187``;
SURVEY §3.5).  Three state kinds are used here instead:

``hist``    exact histogram ``int64 [C, 2, 16384]`` of (class, label, score-code) for bf16/fp16 scores
            (``csrc/classification.hip: curve_hist_update``).  Fixed size -> all-reduced by RCCL instead of
            all-gathered; AUROC / AP for *all* classes come out of one kernel (``curve_hist_reduce``) with no
            per-class loop.  Exact: code order == value order and every distinct score keeps its own bin.
``samples`` ``(preds [N, C], labels [N, C], valid [N, C])`` for fp32/fp64 scores.  On the GPU every class is sorted
            by the hand-written segmented radix sort with a fused tie-group scan (``csrc/radix.hip``, ``sorted_scores``
            / ``sorted_curve_points``: AUROC, AP and curve points at any size, no ATen sort); on the CPU all classes
            are sorted at once with one vectorised tie pass; no per-class loop for AUROC/AP either way.
``binned``  the reference's multi-threshold confusion matrix ``[T, C, 2, 2]`` (``binned_curve_update``).

Curve *points* (distinct thresholds with cumulative tps/fps) are produced per class only when a caller asks
for the curves themselves (PR-curve / ROC outputs are ragged lists by API).
"""
from typing import List, Optional, Tuple, Union

import torch
from torch import Tensor

from torchmetrics_forked_amd import ops
from torchmetrics_forked_amd.ops import classification as cls_ops
from torchmetrics_forked_amd.ops.sort import argsort as _argsort, sort as _sort

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
    if preds.device.type == "cpu" and preds.is_floating_point() and ops.load():
        # host op: per-column radix sort + one tie-group scan (csrc/host_curve.cpp), columns in parallel
        out = torch.ops.tmx.curve_scores_host(preds.detach(), labels, valid)
        return out[:, 0], out[:, 1], out[:, 2], out[:, 3]
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


# ---------------------------------------------------------------------------------------------------------
# GPU fp32 / fp64: segmented radix sort + fused scan (csrc/radix.hip)
# ---------------------------------------------------------------------------------------------------------
_SORT_MAX_ELEMS = 1 << 31  # keys per launch (classes are processed in groups above this)


def _sorted_inputs(preds: Union[Tensor, "ColumnChunks"], target: Tensor, task: str) -> Optional[Tuple[List[Tensor], Tensor, int]]:
    """(chunks [S, n_k], int64 target, task code) for the radix route, or None (CPU / 16-bit / no native library)."""
    if isinstance(preds, ColumnChunks):
        chunks = list(preds.cols)
    else:
        if preds.dtype not in (torch.float32, torch.float64):
            return None
        p2 = preds.reshape(-1, 1) if task == "binary" else preds
        chunks = [p2.t()]
    sample = chunks[0]
    if not (sample.is_cuda and sample.dtype in (torch.float32, torch.float64) and ops.use_native(sample)):
        return None
    t = target.long()
    if task == "multiclass":
        return chunks, t.reshape(-1).contiguous(), 0
    return chunks, t.reshape(chunks[0].shape[1] if task == "binary" else t.shape[0], -1).contiguous(), 1


def _class_groups(chunks: List[Tensor]) -> List[Tuple[int, int]]:
    S = chunks[0].shape[0]
    n = sum(c.shape[1] for c in chunks)
    per = max(1, min(S, _SORT_MAX_ELEMS // max(n, 1)))
    return [(s0, min(S, s0 + per)) for s0 in range(0, S, per)]


def _group_target(t: Tensor, code: int, s0: int, s1: int) -> Tensor:
    """Target of the class group [s0, s1): multiclass ids shifted so class s0 is segment 0; label columns sliced."""
    if code == 0:
        return t if s0 == 0 else (t - s0).contiguous()
    return t if (s0 == 0 and s1 == t.shape[1]) else t[:, s0:s1].contiguous()


def sorted_scores(
    preds: Union[Tensor, "ColumnChunks"], target: Tensor, task: str, ignore_index: Optional[int]
) -> Optional[Tensor]:
    """(auroc, ap, P, N) ``[S, 4]`` float64 per class / label from GPU fp32 / fp64 samples, or None off the GPU."""
    prep = _sorted_inputs(preds, target, task)
    if prep is None:
        return None
    chunks, t, code = prep
    if chunks[0].shape[1] == 0 and len(chunks) == 1:
        return None
    ii = ignore_index if task == "multilabel" else None
    outs = []
    for s0, s1 in _class_groups(chunks):
        outs.append(cls_ops.curve_sorted([c[s0:s1] for c in chunks], _group_target(t, code, s0, s1), code, ii, False)[0])
    return torch.cat(outs) if len(outs) > 1 else outs[0]


def sorted_curve_points(
    preds: Union[Tensor, "ColumnChunks"], target: Tensor, task: str, ignore_index: Optional[int]
) -> Optional[List[Tuple[Tensor, Tensor, Tensor]]]:
    """Per class / label: (fps, tps, thresholds) at every distinct score (descending) from GPU fp32 / fp64 samples."""
    prep = _sorted_inputs(preds, target, task)
    if prep is None:
        return None
    chunks, t, code = prep
    ii = ignore_index if task == "multilabel" else None
    out: List[Tuple[Tensor, Tensor, Tensor]] = []
    for s0, s1 in _class_groups(chunks):
        _, counts, fps, tps, thr = cls_ops.curve_sorted([c[s0:s1] for c in chunks], _group_target(t, code, s0, s1), code, ii, True)
        if ii is not None and fps.numel():
            # groups made only of ignored samples (kept by the kernel) are not thresholds of the reference
            seg = torch.repeat_interleave(torch.arange(counts.numel(), device=fps.device), counts, output_size=fps.numel())
            first = torch.ones_like(seg, dtype=torch.bool)
            first[1:] = seg[1:] != seg[:-1]
            prev_f = torch.where(first, torch.zeros_like(fps), fps.roll(1))
            prev_t = torch.where(first, torch.zeros_like(tps), tps.roll(1))
            keep = (fps != prev_f) | (tps != prev_t)
            counts = torch.bincount(seg[keep], minlength=counts.numel())
            fps, tps, thr = fps[keep], tps[keep], thr[keep]
        sizes = counts.tolist()
        out.extend(zip(torch.split(fps, sizes), torch.split(tps, sizes), torch.split(thr, sizes)))
    return out


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
        pos_rows = None  # sorted below, only when the anchored route is taken
    else:
        p2 = preds.reshape(-1, 1) if task == "binary" else preds
        if task == "binary" and cls_ops.count_exceeds(target, 1, cls_ops.ANCHOR_MAX_POS) > cls_ops.ANCHOR_MAX_POS:
            return None  # decided by a capped count (stops reading once past the cap): no [N] compare + reduce
        lab = (target.reshape(p2.shape) == 1).t()
        C = p2.shape[1]
        counts = lab.sum(1)  # the positions of the positives only when the anchored route is taken (below)
        pos_rows = None
        preds = p2
    max_pos = int(counts.max()) if counts.numel() else 0
    if max_pos > cls_ops.ANCHOR_MAX_POS:
        return None
    if pos_rows is None:
        pos_rows = _argsort(t) if task == "multiclass" else lab.nonzero(as_tuple=True)[1]
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
        sp, order = _sort(preds, descending=True) if preds.dim() == 1 else torch.sort(preds, descending=True)
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
        sv, order = _sort(cols, descending=True)
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

