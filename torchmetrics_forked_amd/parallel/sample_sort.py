"""Sample-sharded compute for rank- and contingency-based metrics (VERDICT r2 "next round" #8).

The reference all-gathers every sample of ``SpearmanCorrCoef`` and of the clustering metrics to every rank and
recomputes the whole metric everywhere (``TF/regression/spearman.py:23-55`` ranks all samples on every rank,
``TF/clustering/utils.py:119-176`` builds the contingency table of all samples on every rank).  With
``sharded_compute=True`` under DDP:

* **Spearman** — a distributed sample sort: every rank proposes splitters from its sorted local values (one small
  uneven all-gather), values are routed to the rank that owns their value range with one ``all_to_all`` (equal values
  always land on one rank, so tie groups are never split), each owner ranks its range (average ranks of ties) and
  offsets by the sizes of the lower ranges, and the ranks travel back to the rows they came from with a second
  ``all_to_all``.  The correlation then needs three all-reduced sums of centred ranks (the mean of average ranks is
  exactly (n + 1) / 2).  Traffic: each sample twice, against world x every sample for the all-gather.
* **Extrinsic clustering** (MI, NMI, AMI, RI, ARI, FMI, homogeneity / completeness / V-measure) — every metric is a
  function of the contingency table: ranks agree on the union of cluster labels (small all-gathers of the unique
  labels), count their own samples into the global ``[K_target, K_pred]`` table and all-reduce it.  No sample
  leaves its rank.
"""
from typing import List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist
from torch import Tensor

from torchmetrics_forked_amd.parallel.shard import all_reduce_sum, exchange_rows
from torchmetrics_forked_amd.parallel.sync import _world
from torchmetrics_forked_amd.utilities.distributed import gather_all_tensors
from torchmetrics_forked_amd.ops.sort import argsort as _argsort, sort as _sort

_SPLITTER_SAMPLES = 64  # per rank and per peer rank


def _rank(group: Optional[object]) -> int:
    return dist.get_rank(group) if group is not None else dist.get_rank()


def _local_average_ranks(sorted_vals: Tensor) -> Tensor:
    """1-based average ranks of an ascending-sorted 1-D tensor (ties share the mean of their positions)."""
    n = sorted_vals.numel()
    if n == 0:
        return torch.zeros(0, dtype=torch.float64, device=sorted_vals.device)
    new = torch.ones(n, dtype=torch.bool, device=sorted_vals.device)
    new[1:] = sorted_vals[1:] != sorted_vals[:-1]
    gid = torch.cumsum(new, 0) - 1
    counts = torch.bincount(gid)
    ends = torch.cumsum(counts, 0)
    avg = (ends - counts + 1 + ends).to(torch.float64) / 2
    return avg[gid]


def _owners(x: Tensor, group: Optional[object]) -> Tensor:
    """Owner rank of every local value: ``world - 1`` splitters are quantiles of evenly spaced samples of every
    rank's sorted values (one small uneven all-gather); equal values always get the same owner and owners are
    ordered by value (rank r owns a range entirely below rank r + 1's)."""
    world = _world(group)
    n_local = x.numel()
    srt = _sort(x)[0]
    k = min(n_local, _SPLITTER_SAMPLES * world)
    pick = srt[torch.linspace(0, n_local - 1, k, device=x.device).round().long()] if k else srt[:0]
    # exchanged as float64 so that ranks without samples (no dtype of their own) take part in the same collective;
    # every rank casts the same splitters back, so equal values still share an owner
    gathered = gather_all_tensors(pick.to(torch.float64).contiguous(), group)
    merged = _sort(torch.cat([t.to(x.device) for t in gathered]))[0].to(x.dtype)
    if merged.numel() == 0:
        return torch.zeros(n_local, dtype=torch.long, device=x.device)
    q = torch.linspace(0, merged.numel() - 1, world + 1, device=x.device)[1:-1].round().long()
    return torch.searchsorted(merged[q].contiguous(), x.contiguous(), right=True)


def _route(x: Tensor, extra: Sequence[Tensor], group: Optional[object]) -> List[Tensor]:
    """Send ``x`` (and row-aligned ``extra`` columns) to the owners of their value ranges; returns the received
    ``[x, *extra]`` on ``x``'s device."""
    owner = _owners(x, group)
    # a rank without samples sends None columns: it adopts the dtypes of the ranks that have data
    cols: List[Optional[Tensor]] = [c if x.numel() else None for c in (x, *extra)]
    recv, _ = exchange_rows(cols, owner, group)
    return [t.to(x.device) for t in recv]


def _range_offset(n_owned: int, group: Optional[object], device: torch.device) -> int:
    """Number of values owned by lower ranks (= global position of this rank's first value)."""
    world, me = _world(group), _rank(group)
    sizes = torch.zeros(world, dtype=torch.long, device=device)
    sizes[me] = n_owned
    return int(all_reduce_sum(sizes, group)[:me].sum())


def global_average_ranks(x: Tensor, group: Optional[object] = None) -> Tensor:
    """Average rank (1-based, float64) of every local value of ``x`` among the values of ALL ranks (see module)."""
    me = _rank(group)
    x = x.reshape(-1)
    n_local = x.numel()
    # 1-2) route every value (with its origin) to the owner of its value range
    src_idx = torch.arange(n_local, device=x.device)
    vals, idx, src = _route(x, [src_idx, torch.full((n_local,), me, dtype=torch.long, device=x.device)], group)
    # 3) rank the owned range, offset by the sizes of the lower ranges
    offset = _range_offset(vals.numel(), group, x.device)
    order = _argsort(vals)
    ranks = torch.empty(vals.numel(), dtype=torch.float64, device=x.device)
    ranks[order] = _local_average_ranks(vals[order]) + offset
    # 4) ranks back to the rows they came from
    back, _ = exchange_rows([ranks, idx], src, group)
    out = torch.empty(n_local, dtype=torch.float64, device=x.device)
    out[back[1].to(x.device).long()] = back[0].to(x.device)
    return out


def sharded_spearman(preds: Tensor, target: Tensor, group: Optional[object] = None, eps: float = 1e-6) -> Tensor:
    """Spearman correlation of the samples of all ranks without gathering them (``preds`` / ``target`` [n] or
    [n, D] local samples); same formula as ``_spearman_corrcoef_compute`` on the concatenated samples."""
    dtype = preds.dtype if preds.is_floating_point() else torch.float32
    d = 1 if preds.ndim == 1 else preds.shape[1]
    p2 = preds.reshape(preds.shape[0], d)
    t2 = target.reshape(target.shape[0], d)
    n = float(all_reduce_sum(torch.tensor([p2.shape[0]], dtype=torch.float64, device=preds.device), group)[0])
    mean = (n + 1.0) / 2.0
    sums = []
    for d in range(p2.shape[1]):
        rp = global_average_ranks(p2[:, d], group) - mean
        rt = global_average_ranks(t2[:, d], group) - mean
        sums.append(torch.stack([(rp * rt).sum(), (rp * rp).sum(), (rt * rt).sum()]))
    tot = all_reduce_sum(torch.stack(sums), group)
    cov, vp, vt = tot[:, 0] / n, tot[:, 1] / n, tot[:, 2] / n
    corr = (cov / (torch.sqrt(vp) * torch.sqrt(vt) + eps)).clamp(-1.0, 1.0).to(dtype)
    return corr[0] if preds.ndim == 1 else corr


def _greater_in_lower_ranges(y: Tensor, xr: Tensor, world: int) -> int:
    """#{(a, b): y_a > y_b and xr_a < xr_b} among the given rows (one owner's y range)."""
    n = y.numel()
    if n < 2:
        return 0
    order = _argsort(y)
    ys, rs = y[order], xr[order].long()
    new = torch.ones(n, dtype=torch.bool, device=y.device)
    new[1:] = ys[1:] != ys[:-1]
    gid = torch.cumsum(new, 0) - 1
    ends = torch.cumsum(torch.bincount(gid), 0)
    onehot = torch.nn.functional.one_hot(rs, world).long()
    suffix = torch.cat([onehot.flip(0).cumsum(0).flip(0), torch.zeros(1, world, dtype=torch.long, device=y.device)])
    greater = suffix[ends[gid]]  # per row: counts (per x range) of rows with a strictly larger y
    below = greater.cumsum(1).gather(1, rs[:, None]) - greater.gather(1, rs[:, None])
    return int(below.sum())


def sharded_kendall_stats(x: Tensor, y: Tensor, group: Optional[object] = None) -> Tuple[Tensor, ...]:
    """Kendall pair / tie statistics of the samples of all ranks for one output column, in the layout of
    ``functional/regression/kendall._column_stats`` plus the global sample count.

    Discordant pairs (x_a < x_b, y_a > y_b) split into three disjoint kinds after routing rows by x range and then by
    y range: pairs inside one x range (local lexicographic inversion count), pairs in different x ranges and
    different y ranges (from the all-reduced [x range, y range] occupancy matrix), and pairs in different x ranges
    but one y range (counted by that y range's owner).  Tie groups never straddle owners, so run-length tie
    statistics are owner-local sums."""
    from torchmetrics_forked_amd.functional.regression.kendall import _count_inversions, _joint_run_lengths, _run_lengths

    world, me = _world(group), _rank(group)
    dev = x.device
    # by x range: inversions inside the range, x ties, joint ties
    xv, yv = _route(x.reshape(-1), [y.reshape(-1)], group)
    oy = _argsort(yv)
    ox = _argsort(xv[oy])
    order = oy[ox]
    xs, ys = xv[order], yv[order]
    dis_local = int(_count_inversions(ys)) if xs.numel() > 1 else 0
    tx = _run_lengths(xs).double() if xs.numel() else torch.zeros(0, dtype=torch.float64, device=dev)
    txy = _joint_run_lengths(xs, ys).double() if xs.numel() else torch.zeros(0, dtype=torch.float64, device=dev)
    # by y range: y ties, same-y-range cross pairs, occupancy
    y2, xr2 = _route(ys, [torch.full((ys.numel(),), me, dtype=torch.long, device=dev)], group)
    ty = _run_lengths(_sort(y2)[0]).double() if y2.numel() else torch.zeros(0, dtype=torch.float64, device=dev)
    dis_same_y = _greater_in_lower_ranges(y2, xr2, world)
    occ = torch.zeros(world, world, dtype=torch.long, device=dev)
    occ[:, me] = torch.bincount(xr2.long(), minlength=world)[:world] if xr2.numel() else 0
    ints = all_reduce_sum(torch.cat([occ.reshape(-1), torch.tensor([dis_local + dis_same_y, xs.numel()], device=dev)]), group)
    m = ints[: world * world].reshape(world, world).tolist()
    dis = int(ints[-2]) + sum(
        m[xb][yb] * sum(m[xa][ya] for xa in range(xb) for ya in range(yb + 1, world))
        for xb in range(world) for yb in range(world) if m[xb][yb]
    )
    n = int(ints[-1])
    fl = all_reduce_sum(torch.stack([
        (tx * (tx - 1) / 2).sum(), (tx * (tx - 1) * (tx - 2)).sum(), (tx * (tx - 1) * (2 * tx + 5)).sum(),
        (ty * (ty - 1) / 2).sum(), (ty * (ty - 1) * (ty - 2)).sum(), (ty * (ty - 1) * (2 * ty + 5)).sum(),
        (txy * (txy - 1) / 2).sum(), torch.tensor(float(tx.numel()), dtype=torch.float64, device=dev),
        torch.tensor(float(ty.numel()), dtype=torch.float64, device=dev),
    ]), group)
    n1, p1x, p2x, n2, p1y, p2y, n3, ux, uy = fl.unbind()
    n0 = n * (n - 1) // 2
    con = (n0 - n1 - n2 + n3).round().long() - dis
    return (con, torch.tensor(dis, device=dev), n1, p1x, p2x, n2, p1y, p2y, float(ux), float(uy), n)


MAX_CONTINGENCY = 1 << 24  # cells of the global table; larger label sets fall back to the replicated gather


def global_contingency(preds: Tensor, target: Tensor, group: Optional[object] = None) -> Optional[Tuple[Tensor, int]]:
    """``([K_target, K_pred] int64 contingency of the samples of all ranks, n)``, or None when the label union is too
    large for a dense table (the caller then gathers the samples)."""
    p = preds.reshape(-1).long()
    t = target.reshape(-1).long()
    up = torch.unique(torch.cat([u.to(p.device) for u in gather_all_tensors(torch.unique(p), group)]))
    ut = torch.unique(torch.cat([u.to(t.device) for u in gather_all_tensors(torch.unique(t), group)]))
    kp, kt = up.numel(), ut.numel()
    if kp * kt > MAX_CONTINGENCY:
        return None
    pi = torch.searchsorted(up, p)
    ti = torch.searchsorted(ut, t)
    local = torch.bincount(ti * kp + pi, minlength=kt * kp).reshape(kt, kp) if p.numel() else torch.zeros(kt, kp, dtype=torch.long, device=p.device)
    cont = all_reduce_sum(local.long(), group)
    return cont, int(cont.sum())


def entropy_from_counts(counts: Tensor) -> Tensor:
    """Shannon entropy (nats) of a label distribution given by its counts (``calculate_entropy`` of the labels)."""
    c = counts[counts > 0]
    if c.numel() == 0:
        return torch.tensor(1.0, device=counts.device)
    n = c.sum()
    return -torch.sum(c / n * (torch.log(c) - torch.log(n)))


class SampleShardedMixin:
    """``sharded_compute=True`` under DDP for metrics whose ``cat`` states are samples: sync gathers nothing, it only
    records the process group; ``compute`` (collective on every rank, as after a replicated sync) then runs the
    sharded algorithm over the local samples.  ``unsync`` forgets the group.  A custom ``dist_sync_fn`` keeps the
    replicated gather (it may not be an all-gather)."""

    _sample_shard: Optional[List[object]] = None

    def _sync_dist(self, dist_sync_fn: object = None, process_group: Optional[object] = None) -> None:
        if self.sharded_compute and (dist_sync_fn is None or dist_sync_fn is gather_all_tensors):  # type: ignore[attr-defined]
            self._sample_shard = [process_group or self.process_group]  # type: ignore[attr-defined]
            return
        super()._sync_dist(dist_sync_fn, process_group)  # type: ignore[misc]

    def unsync(self, should_unsync: bool = True) -> None:
        super().unsync(should_unsync)  # type: ignore[misc]
        if should_unsync:
            self._sample_shard = None

    def _leave_batch_mode(self, saved_compute_on_cpu: bool) -> None:
        # forward's batch compute (dist_sync_on_step) syncs without unsync: forget the group with the synced flag, so a
        # later compute that skips the sync takes the local path instead of issuing collectives
        super()._leave_batch_mode(saved_compute_on_cpu)  # type: ignore[misc]
        self._sample_shard = None

    def _local_samples(self, *names: str, empty_dtype: torch.dtype = torch.float32) -> List[Tensor]:
        """This rank's concatenated sample states (empty rank: a length-0 tensor of ``empty_dtype``)."""
        from torchmetrics_forked_amd.utilities.data import dim_zero_cat

        out = []
        for name in names:
            val = getattr(self, name)
            if isinstance(val, list) and not val:
                out.append(torch.zeros(0, dtype=empty_dtype, device=self.device))  # type: ignore[attr-defined]
            else:
                out.append(dim_zero_cat(val))
        return out


__all__: List[str] = [
    "SampleShardedMixin", "global_average_ranks", "sharded_spearman", "sharded_kendall_stats", "global_contingency", "entropy_from_counts",
]
