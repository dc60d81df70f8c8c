"""Retrieval base (API parity: reference ``retrieval/base.py:25-155``).

States are the reference's three ``None``-reduced lists (indexes / preds / target), so ``state_dict`` and the
rank-interleaved gather order match.  ``compute`` scores every query in one segmented pass (``_grouped``)
instead of a host loop over queries.
"""
from abc import ABC
from typing import Any, List, Optional, Sequence, Union

import torch
import torch.distributed as dist
from torch import Tensor, tensor

from torchmetrics_forked_amd.functional.retrieval._grouped import Grouped
from torchmetrics_forked_amd.metric import Metric
from torchmetrics_forked_amd.utilities.checks import _check_retrieval_inputs
from torchmetrics_forked_amd.utilities.data import dim_zero_cat
from torchmetrics_forked_amd.utilities.plot import _AX_TYPE, _PLOT_OUT_TYPE


class RetrievalMetric(Metric, ABC):
    is_differentiable: bool = False
    higher_is_better: bool = True
    full_state_update: bool = False
    indexes: List[Tensor]
    preds: List[Tensor]
    target: List[Tensor]
    _empty_on_negatives: bool = False  # FallOut: a query is "empty" when it has no negative document

    def __init__(self, empty_target_action: str = "neg", ignore_index: Optional[int] = None, **kwargs: Any) -> None:
        super().__init__(**kwargs)
        self.allow_non_binary_target = False
        options = ("error", "skip", "neg", "pos")
        if empty_target_action not in options:
            raise ValueError(f"Argument `empty_target_action` received a wrong value `{empty_target_action}`.")
        self.empty_target_action = empty_target_action
        if ignore_index is not None and not isinstance(ignore_index, int):
            raise ValueError("Argument `ignore_index` must be an integer or None.")
        self.ignore_index = ignore_index
        self.add_state("indexes", default=[], dist_reduce_fx=None)
        self.add_state("preds", default=[], dist_reduce_fx=None)
        self.add_state("target", default=[], dist_reduce_fx=None)

    def update(self, preds: Tensor, target: Tensor, indexes: Tensor) -> None:
        if indexes is None:
            raise ValueError("Argument `indexes` cannot be None")
        indexes, preds, target = _check_retrieval_inputs(
            indexes,
            preds,
            target,
            allow_non_binary_target=self.allow_non_binary_target,
            ignore_index=self.ignore_index,
            sink=self._validation_sink(target),
        )
        self.indexes.append(indexes)
        self.preds.append(preds)
        self.target.append(target)

    # ------------------------------------------------------------------------------------- sharded compute
    # ``sharded_compute=True`` under DDP: queries are owned by rank ``index mod world``; sync sends every row to its
    # owner with one all_to_all per state (parallel/shard.py) instead of all-gathering everything everywhere, each
    # rank scores only its queries, and the mean over queries is one small all-reduce of (sum, count[, error flag]).
    _shard_group: Optional[Any] = None
    _sharded_active: bool = False  # set between a sharded sync and the matching unsync (the group may be None)

    def _sync_dist(self, dist_sync_fn: Any = None, process_group: Optional[Any] = None) -> None:
        from torchmetrics_forked_amd.utilities.distributed import gather_all_tensors

        if not self.sharded_compute or (dist_sync_fn is not None and dist_sync_fn is not gather_all_tensors):
            super()._sync_dist(dist_sync_fn, process_group)
            return
        from torchmetrics_forked_amd.parallel.shard import exchange_rows

        group = process_group or self.process_group
        world = dist.get_world_size(group) if group is not None else dist.get_world_size()
        have = len(self.indexes) > 0
        idx = dim_zero_cat(self.indexes) if have else None
        cols = [idx, dim_zero_cat(self.preds) if have else None, dim_zero_cat(self.target) if have else None]
        owner = idx.remainder(world) if have else torch.zeros(0, dtype=torch.long, device=self.device)
        (r_idx, r_preds, r_target), _ = exchange_rows(cols, owner, group)
        dev = self.device
        self.indexes, self.preds, self.target = [r_idx.to(dev)], [r_preds.to(dev)], [r_target.to(dev)]
        self._shard_group = group
        self._sharded_active = True

    def unsync(self, should_unsync: bool = True) -> None:
        super().unsync(should_unsync)
        if should_unsync:
            self._shard_group = None
            self._sharded_active = False

    def _sharded_mean(self, values: Tensor, empty: Tensor, out_dtype: torch.dtype, fill_shape: Sequence[int] = ()) -> Tensor:
        """Mean over the queries of all ranks from this rank's per-query values (empty-target policy applied
        globally: "error" raises on every rank if any rank owns an empty query)."""
        from torchmetrics_forked_amd.parallel.shard import all_reduce_sum

        group = self._shard_group
        if self.empty_target_action == "error":
            flag = all_reduce_sum(empty.any().reshape(1).to(torch.float64), group)
            if float(flag) > 0:
                kind = "negative" if self._empty_on_negatives else "positive"
                raise ValueError(f"`compute` method was provided with a query with no {kind} target.")
        values = self._apply_empty_action(values, empty, fill_shape)
        part = torch.cat([values.to(torch.float64).reshape(values.shape[0], -1).sum(0),
                          torch.tensor([float(values.shape[0])], dtype=torch.float64, device=values.device)])
        tot = all_reduce_sum(part, group)
        n = tot[-1]
        width = int(torch.tensor(fill_shape).prod()) if fill_shape else 1
        if float(n) == 0:
            return torch.zeros(fill_shape, dtype=out_dtype, device=values.device) if fill_shape else torch.tensor(0.0, dtype=out_dtype, device=values.device)
        mean = (tot[:width] / n).to(out_dtype)
        return mean.reshape(fill_shape) if fill_shape else mean[0]

    def _grouped(self) -> Grouped:
        return Grouped(dim_zero_cat(self.preds), dim_zero_cat(self.target), dim_zero_cat(self.indexes))

    def _empty_queries(self, g: Grouped) -> Tensor:
        if self._empty_on_negatives:
            return g.seg_sum((g.target <= 0).float()) == 0
        return g.seg_sum(g.target.float()) == 0

    def _apply_empty_action(self, values: Tensor, empty: Tensor, fill_shape: Sequence[int] = ()) -> Tensor:
        if self.empty_target_action == "error" and bool(empty.any()):
            kind = "negative" if self._empty_on_negatives else "positive"
            raise ValueError(f"`compute` method was provided with a query with no {kind} target.")
        mask = empty.reshape(-1, *([1] * len(fill_shape)))
        if self.empty_target_action == "pos":
            return torch.where(mask, torch.ones_like(values), values)
        if self.empty_target_action == "neg":
            return torch.where(mask, torch.zeros_like(values), values)
        if self.empty_target_action == "skip":
            return values[~empty]
        return values

    def compute(self) -> Tensor:
        preds = dim_zero_cat(self.preds)
        g = self._grouped()
        if self._sharded_active:
            return self._sharded_mean(self._per_query(g).to(preds.dtype), self._empty_queries(g), preds.dtype)
        values = self._apply_empty_action(self._per_query(g).to(preds.dtype), self._empty_queries(g))
        return values.mean() if values.numel() else tensor(0.0).to(preds)

    def _per_query(self, g: Grouped) -> Tensor:
        """Metric value of every query, ``[Q]`` (subclasses)."""
        raise NotImplementedError

    def _metric(self, preds: Tensor, target: Tensor) -> Tensor:
        """Single-query metric (reference hook; kept for API compatibility)."""
        return self._per_query(Grouped(preds, target))[0]

    def plot(self, val: Optional[Union[Tensor, Sequence[Tensor]]] = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:
        return self._plot(val, ax)
