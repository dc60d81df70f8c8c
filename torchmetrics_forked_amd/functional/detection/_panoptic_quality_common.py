"""Panoptic quality statistics (API parity: reference ``functional/detection/_panoptic_quality_common.py``).

The reference walks Python dicts of segment "colors" per sample.  Here the whole batch is processed with
device-side tensor ops and no per-segment host loop:

1. every point gets a ``(sample, category index, instance)`` key (stuff instances zeroed, unknown -> void);
2. ``unique`` over the keys gives dense segment ids + areas for predictions and targets;
3. ``unique`` over ``pred_seg * n_target_segs + target_seg`` gives every overlapping pair and its intersection;
4. void overlaps, IoUs (fp32, as the reference's integer-tensor division), the >0.5 matching (unique by
   construction), false positives / negatives and the modified-PQ stuff terms are all segment-parallel
   scatter ops into per-category ``[K]`` accumulators.
"""
from typing import Collection, Dict, Optional, Set, Tuple

import torch
from torch import Tensor

from torchmetrics_forked_amd import ops

from torchmetrics_forked_amd.utilities.prints import rank_zero_warn


def _parse_categories(things: Collection[int], stuffs: Collection[int]) -> Tuple[Set[int], Set[int]]:
    things_parsed = set(things)
    if len(things_parsed) < len(things):
        rank_zero_warn("The provided `things` categories contained duplicates, which have been removed.", UserWarning)
    stuffs_parsed = set(stuffs)
    if len(stuffs_parsed) < len(stuffs):
        rank_zero_warn("The provided `stuffs` categories contained duplicates, which have been removed.", UserWarning)
    if not all(isinstance(v, int) for v in things_parsed):
        raise TypeError(f"Expected argument `things` to contain `int` categories, but got {things}")
    if not all(isinstance(v, int) for v in stuffs_parsed):
        raise TypeError(f"Expected argument `stuffs` to contain `int` categories, but got {stuffs}")
    if things_parsed & stuffs_parsed:
        raise ValueError(f"Expected arguments `things` and `stuffs` to have distinct keys, but got {things} and {stuffs}")
    if not (things_parsed | stuffs_parsed):
        raise ValueError("At least one of `things` and `stuffs` must be non-empty.")
    return things_parsed, stuffs_parsed


def _validate_inputs(preds: Tensor, target: Tensor) -> None:
    if not isinstance(preds, Tensor):
        raise TypeError(f"Expected argument `preds` to be of type `torch.Tensor`, but got {type(preds)}")
    if not isinstance(target, Tensor):
        raise TypeError(f"Expected argument `target` to be of type `torch.Tensor`, but got {type(target)}")
    if preds.shape != target.shape:
        raise ValueError(
            f"Expected argument `preds` and `target` to have the same shape, but got {preds.shape} and {target.shape}"
        )
    if preds.dim() < 3:
        raise ValueError(
            "Expected argument `preds` to have at least one spatial dimension (B, *spatial_dims, 2), "
            f"got {preds.shape}"
        )
    if preds.shape[-1] != 2:
        raise ValueError(
            "Expected argument `preds` to have exactly 2 channels in the last dimension (category, instance), "
            f"got {preds.shape} instead"
        )


def _get_void_color(things: Set[int], stuffs: Set[int]) -> Tuple[int, int]:
    return 1 + max([0, *things, *stuffs]), 0


def _get_category_id_to_continuous_id(things: Set[int], stuffs: Set[int]) -> Dict[int, int]:
    """Things first, then stuffs, each in set iteration order (same layout as the reference's state vectors)."""
    out = {t: i for i, t in enumerate(things)}
    out.update({s: i + len(things) for i, s in enumerate(stuffs)})
    return out


def _isin(arr: Tensor, values: Collection[int]) -> Tensor:
    if len(values) == 0:
        return torch.zeros_like(arr, dtype=torch.bool)
    return torch.isin(arr, torch.tensor(sorted(values), dtype=arr.dtype, device=arr.device))


def _prepocess_inputs(
    things: Set[int], stuffs: Set[int], inputs: Tensor, void_color: Tuple[int, int], allow_unknown_category: bool
) -> Tensor:
    """Flatten to ``[B, P, 2]``; zero stuff instance ids; map unknown categories to the void color."""
    out = torch.flatten(inputs.detach(), 1, -2).clone()
    cat = out[..., 0]
    is_stuff = _isin(cat, stuffs)
    is_thing = _isin(cat, things)
    known = is_stuff | is_thing
    if not allow_unknown_category and not bool(known.all()):
        raise ValueError(f"Unknown categories found: {out[~known]}")
    out[..., 1] = torch.where(is_stuff, torch.zeros_like(out[..., 1]), out[..., 1])
    void = out.new_tensor(void_color)
    out = torch.where(known[..., None], out, void)
    return out


def _segments(flat: Tensor, cat_idx: Tensor) -> Tuple[Tensor, Tensor, Tensor]:
    """Dense segment ids per point, plus per-segment (category index, area)."""
    b, p = flat.shape[:2]
    sample = torch.arange(b, device=flat.device).repeat_interleave(p)
    keys = torch.stack([sample, cat_idx.reshape(-1), flat[..., 1].reshape(-1).long()], 1)
    uniq, inv, area = torch.unique(keys, dim=0, return_inverse=True, return_counts=True)
    return inv, uniq[:, 1], area


def _segments_native(fp: Tensor, ft: Tensor, id_t: Tensor, cont_t: Tensor, k: int) -> Optional[Tuple[Tuple[Tensor, ...], ...]]:
    """GPU: one csrc/panoptic.hip pass packs (image, category index, instance) of every pixel into an ordered int64
    key; segments come from a 1-D unique of the keys (same order as the row unique).  ``None`` -> row path."""
    if not (fp.is_cuda and fp.dtype == torch.long and ft.dtype == torch.long and ops.use_native(fp)):
        return None
    if fp.shape[0] >= 32768 or k >= 65535 or id_t.numel() > 4096:
        return None
    pkey, tkey, overflow = torch.ops.tmx.panoptic_segment_keys(fp, ft, id_t, cont_t)
    if int(overflow.item()):
        return None
    out = []
    for key in (pkey, tkey):
        uniq, inv, area = torch.unique(key, sorted=True, return_inverse=True, return_counts=True)
        out.append((inv, (uniq >> 32) & 0xFFFF, area))
    return tuple(out)


def _panoptic_quality_update(
    flatten_preds: Tensor,
    flatten_target: Tensor,
    cat_id_to_continuous_id: Dict[int, int],
    void_color: Tuple[int, int],
    modified_metric_stuffs: Optional[Set[int]] = None,
) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    """Per-category ``(iou_sum [K] fp64, tp [K] int32, fp [K] int32, fn [K] int32)`` for a ``[B, P, 2]`` batch."""
    device = flatten_preds.device
    k = len(cat_id_to_continuous_id)
    iou_sum = torch.zeros(k, dtype=torch.double, device=device)
    tp = torch.zeros(k, dtype=torch.int, device=device)
    fp = torch.zeros(k, dtype=torch.int, device=device)
    fn = torch.zeros(k, dtype=torch.int, device=device)
    if flatten_preds.numel() == 0:
        return iou_sum, tp, fp, fn
    modified = modified_metric_stuffs or set()

    # category id -> continuous index (void and anything unmapped -> k)
    ids = sorted(cat_id_to_continuous_id)
    id_t = torch.tensor(ids, dtype=torch.long, device=device)
    cont_t = torch.tensor([cat_id_to_continuous_id[i] for i in ids] + [k], dtype=torch.long, device=device)
    mod_t = torch.zeros(k + 1, dtype=torch.bool, device=device)
    for c in modified:
        if c in cat_id_to_continuous_id:
            mod_t[cat_id_to_continuous_id[c]] = True

    def to_idx(cat: Tensor) -> Tensor:
        cat = cat.long().contiguous()
        pos = torch.searchsorted(id_t, cat).clamp_max(len(ids) - 1)
        hit = id_t[pos] == cat
        return torch.where(hit, cont_t[pos], torch.full_like(cat, k))

    segs = _segments_native(flatten_preds, flatten_target, id_t, cont_t, k)
    if segs is not None:
        (p_inv, p_cat, p_area), (t_inv, t_cat, t_area) = segs
    else:
        p_inv, p_cat, p_area = _segments(flatten_preds, to_idx(flatten_preds[..., 0]))
        t_inv, t_cat, t_area = _segments(flatten_target, to_idx(flatten_target[..., 0]))
    n_p, n_t = p_cat.numel(), t_cat.numel()
    pair, inter_all = torch.unique(p_inv * n_t + t_inv, return_counts=True)
    ps, ts = pair // n_t, pair % n_t
    p_void, t_void = p_cat == k, t_cat == k

    pred_void_area = torch.zeros(n_p, dtype=torch.long, device=device)
    sel = t_void[ts]
    pred_void_area.index_add_(0, ps[sel], inter_all[sel])
    void_target_area = torch.zeros(n_t, dtype=torch.long, device=device)
    sel = p_void[ps]
    void_target_area.index_add_(0, ts[sel], inter_all[sel])

    cand = (~t_void[ts]) & (p_cat[ps] == t_cat[ts])
    a, b, inter = ps[cand], ts[cand], inter_all[cand]
    union = p_area[a] - pred_void_area[a] + t_area[b] - void_target_area[b] - inter
    iou = inter.float() / union.float()
    cat = t_cat[b]
    is_mod = mod_t[cat]
    match = (~is_mod) & (iou > 0.5)
    tp += torch.bincount(cat[match], minlength=k + 1)[:k].int()
    iou_sum.index_add_(0, cat[match], iou[match].double())
    mod_hit = is_mod & (iou > 0)
    iou_sum.index_add_(0, cat[mod_hit], iou[mod_hit].double())

    matched_p = torch.zeros(n_p, dtype=torch.bool, device=device)
    matched_p[a[match]] = True
    matched_t = torch.zeros(n_t, dtype=torch.bool, device=device)
    matched_t[b[match]] = True
    fn_mask = (~t_void) & (~matched_t) & (~mod_t[t_cat]) & (void_target_area.float() / t_area.float() <= 0.5)
    fp_mask = (~p_void) & (~matched_p) & (~mod_t[p_cat]) & (pred_void_area.float() / p_area.float() <= 0.5)
    fn += torch.bincount(t_cat[fn_mask], minlength=k + 1)[:k].int()
    fp += torch.bincount(p_cat[fp_mask], minlength=k + 1)[:k].int()
    # modified PQ: stuff "true positives" count the target segments of each modified stuff category
    tp += torch.bincount(t_cat[(~t_void) & mod_t[t_cat]], minlength=k + 1)[:k].int()
    return iou_sum, tp, fp, fn


def _panoptic_quality_compute(iou_sum: Tensor, true_positives: Tensor, false_positives: Tensor, false_negatives: Tensor) -> Tensor:
    denominator = (true_positives + 0.5 * false_positives + 0.5 * false_negatives).double()
    pq = torch.where(denominator > 0.0, iou_sum / denominator, 0.0)
    return torch.mean(pq[denominator > 0])
