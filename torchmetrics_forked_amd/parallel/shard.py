"""State-parallel ("sharded") compute helpers: route rows to the rank that owns them with RCCL
``all_to_all`` instead of all-gathering every row to every rank.

The reference all-gathers the complete ``cat`` states on every rank and then each rank recomputes *everything*
(``retrieval/base.py:114-141`` computes every query on every rank).  With ``sharded_compute=True`` a metric whose
result is a sum / mean over independent groups (queries, classes) instead:

1. derives an owner rank per row (``group_id mod world``),
2. exchanges rows with one ``all_to_all_single`` per state tensor (each rank sends every row exactly once, to one
   rank: total traffic = the data once, against world x the data for an all-gather),
3. computes only the groups it owns, and
4. combines per-group results with a small all-reduce.

Over xGMI (point-to-point links) the all-to-all is link-parallel: every GPU pair exchanges only its share.
Rows arrive grouped by source rank and keep their local order, i.e. the same relative order as the reference's
rank-interleaved gather, so tie-breaking inside a group is unchanged.
"""
from typing import List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist
from torch import Tensor

from torchmetrics_forked_amd.parallel.sync import _collective, _comm_device, _world
from torchmetrics_forked_amd.ops.sort import argsort as _argsort

_DTYPES: Tuple[torch.dtype, ...] = (
    torch.float64, torch.float32, torch.float16, torch.bfloat16, torch.int64, torch.int32, torch.int16, torch.int8,
    torch.uint8, torch.bool,
)


def _code(dtype: torch.dtype) -> int:
    return _DTYPES.index(dtype) if dtype in _DTYPES else 0


def exchange_rows(
    columns: Sequence[Optional[Tensor]], owner: Tensor, group: Optional[object] = None
) -> Tuple[List[Tensor], List[torch.dtype]]:
    """Send row ``i`` of every column to rank ``owner[i]``; returns the rows this rank received (grouped by source
    rank, local order kept) and the agreed dtype of every column.

    ``columns[j]`` may be ``None`` on a rank without data: its dtype and trailing shape are adopted from the ranks
    that have data (one small all-gather of per-rank headers carries the send counts, dtypes and trailing sizes,
    so empty ranks need no prior knowledge).  Columns travel with their own dtype (one all_to_all each)."""
    world = _world(group)
    ncol = len(columns)
    sample = next((c for c in columns if c is not None), None)
    dev = _comm_device(sample if sample is not None else owner, group)
    n_local = 0 if sample is None else sample.shape[0]
    send = torch.bincount(owner.reshape(-1).long().to(dev), minlength=world)[:world] if n_local else torch.zeros(world, dtype=torch.long, device=dev)
    # header: send counts | per column (has, dtype code, trailing numel)
    meta = []
    for c in columns:
        if c is None:
            meta += [0, 0, 0]
        else:
            meta += [1, _code(c.dtype), int(c[0].numel()) if c.dim() > 1 else 1]
    header = torch.cat([send.long(), torch.tensor(meta, dtype=torch.long, device=dev)])
    allh = torch.empty(world, header.numel(), dtype=torch.long, device=dev)
    _collective(dist.all_gather_into_tensor, allh.view(-1), header, what="all_gather(shard headers)", group=group)
    allh_l = allh.tolist()
    rank = dist.get_rank(group) if group is not None else dist.get_rank()
    recv_counts = [allh_l[r][rank] for r in range(world)]
    send_counts = send.tolist()
    dtypes: List[torch.dtype] = []
    widths: List[int] = []
    for j in range(ncol):
        codes = {allh_l[r][world + 3 * j + 1] for r in range(world) if allh_l[r][world + 3 * j]}
        wids = {allh_l[r][world + 3 * j + 2] for r in range(world) if allh_l[r][world + 3 * j]}
        if len(codes) > 1 or len(wids) > 1:
            raise RuntimeError(f"sharded compute: ranks hold column {j} with different dtypes / shapes; cast the inputs to one dtype")
        dtypes.append(_DTYPES[codes.pop()] if codes else torch.float32)
        widths.append(wids.pop() if wids else 1)
    order = _argsort(owner.reshape(-1).long().to(dev)) if n_local else None
    out: List[Tensor] = []
    for j, c in enumerate(columns):
        trail: Tuple[int, ...] = tuple(c.shape[1:]) if c is not None and c.dim() > 1 else ((widths[j],) if widths[j] != 1 else ())
        wire = torch.uint8 if dtypes[j] == torch.bool else dtypes[j]
        src = c[order.to(c.device)].to(dev, wire).contiguous() if (c is not None and n_local) else torch.empty((0, *trail), dtype=wire, device=dev)
        dst = torch.empty((sum(recv_counts), *trail), dtype=wire, device=dev)
        _collective(
            dist.all_to_all_single, dst, src, output_split_sizes=recv_counts, input_split_sizes=send_counts,
            what=f"all_to_all(sharded column {j})", group=group,
        )
        out.append(dst.to(dtypes[j]) if wire != dtypes[j] else dst)
    return out, dtypes


def all_reduce_sum(t: Tensor, group: Optional[object] = None) -> Tensor:
    """Sum of ``t`` over the ranks (on the communication device; returned on ``t``'s device)."""
    dev = _comm_device(t, group)
    buf = t.to(dev).clone()
    _collective(dist.all_reduce, buf, op=dist.ReduceOp.SUM, what="all_reduce(sharded partials)", group=group)
    return buf.to(t.device)


def all_reduce_max(t: Tensor, group: Optional[object] = None) -> Tensor:
    dev = _comm_device(t, group)
    buf = t.to(dev).clone()
    _collective(dist.all_reduce, buf, op=dist.ReduceOp.MAX, what="all_reduce(sharded maxima)", group=group)
    return buf.to(t.device)
