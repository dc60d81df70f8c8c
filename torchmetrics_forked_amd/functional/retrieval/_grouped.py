"""Segmented retrieval engine.

The reference sorts by query id, copies the split sizes to the host and runs a Python loop over queries calling
the per-query functional.  Here all queries are scored at once:

  1. ``gid`` = dense query id (``unique(..., return_inverse=True)``); one lexicographic sort by (gid, -score)
     (two stable sorts);
  2. ``pos`` = rank inside the query = global position - query start;
  3. every metric is a segmented reduction over (gid, pos) with ``index_add`` / ``bincount`` / global cumsums.

All tensors stay on the device; the only host value is the number of queries.  The functional API uses the same
engine with a single query.
"""
from typing import Optional, Tuple

import torch
from torch import Tensor

from torchmetrics_forked_amd import ops
from torchmetrics_forked_amd.ops.sort import argsort as _argsort


class Grouped:
    """Queries laid out contiguously, documents sorted by descending score within each query."""

    def __init__(self, preds: Tensor, target: Tensor, indexes: Optional[Tensor] = None, sort_key: Optional[Tensor] = None) -> None:
        dev = preds.device
        n = preds.numel()
        if indexes is None:
            gid = torch.zeros(n, dtype=torch.long, device=dev)
            self.Q = 1
        else:
            _, gid = torch.unique(indexes, return_inverse=True)
            self.Q = int(gid.max()) + 1 if n else 0
        key = preds if sort_key is None else sort_key
        o1 = _argsort(key, descending=True)
        o2 = _argsort(gid[o1])
        order = o1[o2]
        self.order = order
        self.gid = gid[order]
        self.preds = preds[order]
        self.target = target[order]
        self.sizes = torch.bincount(self.gid, minlength=self.Q)
        self.start = torch.cumsum(self.sizes, 0) - self.sizes
        self.pos = torch.arange(n, device=dev) - self.start[self.gid]
        self.n = n

    # ---------------------------------------------------------------------------------------- primitives
    def seg_sum(self, values: Tensor) -> Tensor:
        out = torch.zeros(self.Q, dtype=values.dtype if values.is_floating_point() else torch.long, device=values.device)
        return out.index_add_(0, self.gid, values if values.is_floating_point() else values.long())

    def seg_cumsum(self, values: Tensor) -> Tensor:
        """Inclusive cumulative sum restarting at every query."""
        c = torch.cumsum(values, 0)
        before = c[self.start] - values[self.start]  # exclusive prefix at each query start
        return c - before[self.gid]

    def k_per_query(self, top_k: Optional[int], adaptive: bool = False) -> Tensor:
        """Per-query cut-off (``None`` -> the query length; ``adaptive`` clamps to the length)."""
        if top_k is None:
            return self.sizes.clone()
        k = torch.full_like(self.sizes, top_k)
        return torch.minimum(k, self.sizes) if adaptive else k

    def in_top(self, k: Tensor) -> Tensor:
        return self.pos < k[self.gid]

    # ---------------------------------------------------------------------------------------- native path
    def stats(self, top_k: Optional[int], adaptive: bool = False, ideal: Optional[Tensor] = None) -> Optional[Tensor]:
        """fp64 ``[Q, 10]`` per-query statistics from ``csrc/retrieval.hip`` (one wave per query): (rel_total,
        neg_total, rel_in_k, neg_in_k, ap_sum, first_rel, rel_in_R, dcg, idcg, k); ``None`` off the GPU."""
        p, t = self.preds, self.target
        if not (p.is_cuda and p.dtype in (torch.float32, torch.float64) and ops.use_native(p)):
            return None
        if t.dtype not in (torch.float32, torch.float64, torch.int64, torch.int32):
            t = t.float() if t.is_floating_point() else t.long()
        ideal = t if ideal is None else ideal.to(t.dtype).contiguous()
        key = (p.device, self.n)
        dtab = _DTAB.get(key)
        if dtab is None:
            disc = 1.0 / torch.log2(torch.arange(self.n, dtype=torch.float64, device=p.device) + 2.0)
            dtab = torch.cat([torch.zeros(1, dtype=torch.float64, device=p.device), torch.cumsum(disc, 0)])
            _DTAB.clear()
            _DTAB[key] = dtab
        return torch.ops.tmx.retrieval_segments(
            p.contiguous(), t.contiguous(), ideal, self.start, self.sizes, -1 if top_k is None else int(top_k), bool(adaptive), dtab
        )


_DTAB: dict = {}  # discount prefix table of the last (device, length)


def _safe_div(num: Tensor, den: Tensor) -> Tensor:
    return torch.where(den > 0, num / den.clamp(min=1e-300), torch.zeros_like(num)).float()


def _binary(target: Tensor) -> Tensor:
    return (target > 0).to(torch.float32)


def per_query_average_precision(g: Grouped, top_k: Optional[int]) -> Tensor:
    st = g.stats(top_k)
    if st is not None:
        return _safe_div(st[:, 4], st[:, 2])
    rel = _binary(g.target) * g.in_top(g.k_per_query(top_k)).float()
    cum = g.seg_cumsum(rel)
    contrib = torch.where(rel > 0, cum / (g.pos + 1).float(), torch.zeros_like(cum))
    n_rel = g.seg_sum(rel)
    return torch.where(n_rel > 0, g.seg_sum(contrib) / n_rel.clamp(min=1), torch.zeros_like(n_rel))


def per_query_reciprocal_rank(g: Grouped, top_k: Optional[int]) -> Tensor:
    st = g.stats(top_k)
    if st is not None:
        return torch.where(st[:, 5] >= 0, 1.0 / (st[:, 5] + 1.0), torch.zeros_like(st[:, 5])).float()
    rel = (g.target > 0) & g.in_top(g.k_per_query(top_k))
    big = torch.full_like(g.pos, g.n + 1)
    first = torch.full((g.Q,), g.n + 1, dtype=torch.long, device=g.pos.device)
    first = first.scatter_reduce(0, g.gid, torch.where(rel, g.pos, big), reduce="amin")
    return torch.where(first <= g.n, 1.0 / (first.float() + 1.0), torch.zeros(g.Q, device=g.pos.device))


def per_query_relevant_in_top(g: Grouped, k: Tensor, negatives: bool = False) -> Tensor:
    t = (g.target <= 0) if negatives else (g.target > 0)
    return g.seg_sum((t & g.in_top(k)).float())


def per_query_precision(g: Grouped, top_k: Optional[int], adaptive_k: bool) -> Tensor:
    st = g.stats(top_k, adaptive=adaptive_k)
    if st is not None:
        return torch.where(st[:, 0] > 0, st[:, 2] / st[:, 9].clamp(min=1), torch.zeros_like(st[:, 2])).float()
    k = g.k_per_query(top_k, adaptive=adaptive_k)
    rel = per_query_relevant_in_top(g, k)
    total = g.seg_sum(_binary(g.target))
    return torch.where(total > 0, rel / k.float(), torch.zeros_like(rel))


def per_query_recall(g: Grouped, top_k: Optional[int]) -> Tensor:
    st = g.stats(top_k)
    if st is not None:
        return _safe_div(st[:, 2], st[:, 0])
    rel = per_query_relevant_in_top(g, g.k_per_query(top_k))
    total = g.seg_sum(_binary(g.target))
    return torch.where(total > 0, rel / total.clamp(min=1), torch.zeros_like(rel))


def per_query_fall_out(g: Grouped, top_k: Optional[int]) -> Tensor:
    st = g.stats(top_k)
    if st is not None:
        return _safe_div(st[:, 3], st[:, 1])
    neg = per_query_relevant_in_top(g, g.k_per_query(top_k), negatives=True)
    total = g.seg_sum((g.target <= 0).float())
    return torch.where(total > 0, neg / total.clamp(min=1), torch.zeros_like(neg))


def per_query_hit_rate(g: Grouped, top_k: Optional[int]) -> Tensor:
    st = g.stats(top_k)
    if st is not None:
        return (st[:, 2] > 0).float()
    return (per_query_relevant_in_top(g, g.k_per_query(top_k)) > 0).float()


def per_query_r_precision(g: Grouped) -> Tensor:
    st = g.stats(None)
    if st is not None:
        return _safe_div(st[:, 6], st[:, 0])
    total = g.seg_sum(_binary(g.target))
    rel = per_query_relevant_in_top(g, total.long())
    return torch.where(total > 0, rel / total.clamp(min=1), torch.zeros_like(rel))


def _discount(pos: Tensor, k: Tensor) -> Tensor:
    d = 1.0 / torch.log2(pos.float() + 2.0)
    return torch.where(pos < k, d, torch.zeros_like(d))


def per_query_ndcg(g: Grouped, top_k: Optional[int]) -> Tensor:
    target = g.target.float()
    if g.preds.is_cuda and g.preds.dtype in (torch.float32, torch.float64) and ops.use_native(g.preds):
        ideal_t = Grouped(target, target, g.gid if g.Q > 1 else None, sort_key=target).target
        st = g.stats(top_k, ideal=ideal_t)
        return torch.where(st[:, 8] == 0, torch.zeros_like(st[:, 7]), st[:, 7] / torch.where(st[:, 8] == 0, torch.ones_like(st[:, 8]), st[:, 8])).float()
    k = g.k_per_query(top_k)[g.gid]
    # tie-averaged DCG: documents with equal score inside a query share the mean gain over their positions
    new = torch.ones(g.n, dtype=torch.bool, device=target.device)
    new[1:] = (g.gid[1:] != g.gid[:-1]) | (g.preds[1:] != g.preds[:-1])
    tie = torch.cumsum(new, 0) - 1
    n_ties = int(tie[-1]) + 1 if g.n else 0
    disc = _discount(g.pos, k)
    t_sum = torch.zeros(n_ties, device=target.device).index_add_(0, tie, target)
    d_sum = torch.zeros(n_ties, device=target.device).index_add_(0, tie, disc)
    cnt = torch.bincount(tie, minlength=n_ties).float()
    tie_gid = torch.zeros(n_ties, dtype=torch.long, device=target.device).scatter_(0, tie, g.gid)
    dcg = torch.zeros(g.Q, device=target.device).index_add_(0, tie_gid, t_sum / cnt * d_sum)
    # ideal DCG: targets sorted descending inside each query (ties irrelevant)
    ideal = Grouped(target, target, g.gid if g.Q > 1 else None, sort_key=target)
    idcg = ideal.seg_sum(ideal.target * _discount(ideal.pos, g.k_per_query(top_k)[ideal.gid]))
    return torch.where(idcg == 0, torch.zeros_like(dcg), dcg / torch.where(idcg == 0, torch.ones_like(idcg), idcg))


def per_query_pr_curve(g: Grouped, max_k: int, adaptive_k: bool) -> Tuple[Tensor, Tensor, Tensor]:
    """Per query ``[Q, max_k]`` precision@k / recall@k and the top-k denominators."""
    dev = g.target.device
    rel = torch.zeros(g.Q, max_k, device=dev)
    keep = g.pos < max_k
    rel.index_put_((g.gid[keep], g.pos[keep]), _binary(g.target)[keep], accumulate=True)
    rel = torch.cumsum(rel, 1)
    ks = torch.arange(1, max_k + 1, device=dev).unsqueeze(0).expand(g.Q, max_k)
    topk = torch.minimum(ks, g.sizes.unsqueeze(1)) if adaptive_k else ks
    total = g.seg_sum(_binary(g.target)).unsqueeze(1)
    return rel / topk.float(), rel / total.clamp(min=1), topk
