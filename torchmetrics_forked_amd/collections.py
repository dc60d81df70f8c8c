"""``MetricCollection`` (API parity: reference ``collections.py:34-660``) with two MI355X-first additions.

1. **Collection-level coalesced, overlapped sync.**  ``compute()`` synchronises the states of *all* members
   (compute-group leaders only, members share state by reference) with coalesced plans
   (:class:`parallel.sync.PendingSyncMany`): one RCCL ``all_reduce`` per (op, dtype) bucket and one packed
   all-gather for list states per member group, instead of each member syncing on its own (reference SURVEY §3.4:
   members re-gather shared tensors).  Members are grouped in compute order up to ~1 MiB of reducible state; every
   group's all-reduces are enqueued up front and a group is waited for only when its first member computes, so
   member ``i``'s compute kernels overlap the transfers of the members after it (reference: blocking per-member
   sync inside each ``compute``, ``collections.py:309-358`` / ``metric.py:423-453``).
2. **Fused update plans.**  Members that consume the same ``(preds, target)`` and advertise a compatible
   ``_fusion_key()`` (e.g. ``MulticlassAUROC`` exact-histogram + ``MulticlassConfusionMatrix`` on the same
   logits) are updated by one fused kernel pass over ``preds`` (:mod:`..ops.fused`), instead of one pass per
   metric.  Compute groups (identical states, reference ``collections.py:200-307``) are still formed after the
   first update.
"""
from collections import OrderedDict
from copy import deepcopy
from typing import Any, Dict, Hashable, Iterable, Iterator, List, Optional, Sequence, Tuple, Union

import torch
from torch import Tensor
from torch.nn import ModuleDict

from torchmetrics_forked_amd.metric import Metric
from torchmetrics_forked_amd.parallel.sync import _REDUCE_OPS as _ALLREDUCED
from torchmetrics_forked_amd.parallel.sync import PendingSyncMany, sync_states_many, sync_timeout
from torchmetrics_forked_amd.utilities.data import _flatten_dict, allclose
from torchmetrics_forked_amd.utilities.plot import _AX_TYPE, _PLOT_OUT_TYPE, plot_single_or_multi_val
from torchmetrics_forked_amd.utilities.prints import rank_zero_warn
from torchmetrics_forked_amd.utilities.validation import forward_scope, host_checks


class MetricCollection(ModuleDict):
    """Chain metrics sharing a call signature; ``update``/``forward``/``compute`` fan out to every member."""

    _modules: Dict[str, Metric]  # type: ignore[assignment]
    _groups: Dict[int, List[str]]

    def __init__(
        self,
        metrics: Union[Metric, Sequence[Metric], Dict[str, Metric]],
        *additional_metrics: Metric,
        prefix: Optional[str] = None,
        postfix: Optional[str] = None,
        compute_groups: Union[bool, List[List[str]]] = True,
    ) -> None:
        super().__init__()
        self.prefix = self._check_arg(prefix, "prefix")
        self.postfix = self._check_arg(postfix, "postfix")
        self._enable_compute_groups = compute_groups
        self._groups_checked: bool = False
        self._state_is_copy: bool = False
        self._fused_plans: Optional[List[Any]] = None
        self.add_metrics(metrics, *additional_metrics)

    # ------------------------------------------------------------------------------------------- update
    @torch.jit.unused
    def forward(self, *args: Any, **kwargs: Any) -> Dict[str, Any]:
        # every member's batch value registers its host checks with one block: one device->host read per forward
        with forward_scope(), host_checks():
            return self._compute_and_reduce("forward", *args, **kwargs)

    def _leaders(self) -> List[str]:
        if self._groups_checked:
            return [cg[0] for cg in self._groups.values()]
        return [str(k) for k in self.keys(keep_base=True)]

    def update(self, *args: Any, **kwargs: Any) -> None:
        """Update every member (only compute-group leaders after the first call), fusing where possible."""
        if self._groups_checked:
            leaders = self._leaders()
            done = self._run_fused_plans(leaders, args, kwargs)
            for name in leaders:
                if name in done:
                    continue
                m0 = getattr(self, name)
                m0.update(*args, **m0._filter_kwargs(**kwargs))
            if self._state_is_copy:
                self._compute_groups_create_state_ref()
                self._state_is_copy = False
        else:
            names = [str(k) for k in self.keys(keep_base=True)]
            done = self._run_fused_plans(names, args, kwargs)
            for name in names:
                if name in done:
                    continue
                m = self._modules[name]
                m.update(*args, **m._filter_kwargs(**kwargs))
            if self._enable_compute_groups:
                self._merge_compute_groups()
                self._compute_groups_create_state_ref()
                self._groups_checked = True

    def _run_fused_plans(self, names: List[str], args: Tuple, kwargs: Dict[str, Any]) -> set:
        from torchmetrics_forked_amd.ops.fused import build_fused_plans

        if self._fused_plans is None:
            self._fused_plans = build_fused_plans(self._modules)
        done: set = set()
        for plan in self._fused_plans:
            members = [n for n in plan.names if n in names]
            if len(members) < 2:
                continue
            done.update(plan.run({n: self._modules[n] for n in members}, args, kwargs))
        return done

    def _merge_compute_groups(self) -> None:
        """Merge groups whose leaders hold identical states (O(M^2) comparisons, once)."""
        changed = True
        while changed:
            changed = False
            keys = list(self._groups.keys())
            for i, k1 in enumerate(keys):
                for k2 in keys[i + 1 :]:
                    m1 = getattr(self, self._groups[k1][0])
                    m2 = getattr(self, self._groups[k2][0])
                    if self._equal_metric_states(m1, m2):
                        self._groups[k1].extend(self._groups.pop(k2))
                        changed = True
                        break
                if changed:
                    break
        self._groups = dict(enumerate(self._groups.values()))

    @staticmethod
    def _equal_metric_states(metric1: Metric, metric2: Metric) -> bool:
        if len(metric1._defaults) == 0 or len(metric2._defaults) == 0:
            return False
        if metric1._defaults.keys() != metric2._defaults.keys():
            return False
        for key in metric1._defaults:
            s1, s2 = getattr(metric1, key), getattr(metric2, key)
            if type(s1) != type(s2):  # noqa: E721
                return False
            if isinstance(s1, Tensor):
                if s1.shape != s2.shape or not allclose(s1, s2):
                    return False
            elif isinstance(s1, list):
                if len(s1) != len(s2) or not all(a.shape == b.shape and allclose(a, b) for a, b in zip(s1, s2)):
                    return False
        return True

    def _compute_groups_create_state_ref(self, copy: bool = False) -> None:
        """Point every group member's states at the leader's (or deep-copy them when ``copy``)."""
        if not self._state_is_copy:
            for cg in self._groups.values():
                if len(cg) == 1:  # a singleton group has no members to point at its leader
                    continue
                m0 = getattr(self, cg[0])
                for name in cg[1:]:
                    mi = getattr(self, name)
                    for state in m0._defaults:
                        val = getattr(m0, state)
                        setattr(mi, state, deepcopy(val) if copy else val)
                    mi._update_count = deepcopy(m0._update_count) if copy else m0._update_count
        self._state_is_copy = copy

    # ------------------------------------------------------------------------------------------ compute
    def compute(self) -> Dict[str, Any]:
        # one device->host read for the whole collection: members register their flag checks with this block
        with host_checks():
            synced = self._collection_sync()
            try:
                return self._compute_and_reduce("compute")
            finally:
                self._collection_unsync(synced)

    # reducible bytes per async sync group: members are grouped in compute order until a group carries this much
    # (one coalesced all-reduce per group and dtype); small states stay in one collective, large ones (confusion
    # matrices, FID moments, histograms) get their own so the next member's transfer overlaps this one's compute
    _OVERLAP_GROUP_BYTES = 1 << 20

    def _collection_sync(self) -> List[Tuple[Metric, bool]]:
        """Start syncing every eligible leader (async, grouped); returns (metric, previous _to_sync) to restore.

        The all-reduce buckets of every group are enqueued at once, in member order (the same on every rank); each
        group's states are installed only when its first member computes (``_install_pending``), so the compute
        kernels of earlier members run while later groups' collectives are still in flight on RCCL's stream."""
        self._pending_sync: Dict[int, Any] = {}
        members = list(self._modules.values())
        if not members:
            return []
        leaders = [getattr(self, n) for n in self._leaders()]
        eligible = [
            m
            for m in leaders
            if m._defaults
            and m._to_sync
            and m.dist_sync_fn is None
            and not m._is_synced
            and m._computed is None
            and type(m)._sync_dist is Metric._sync_dist
            and m.distributed_available_fn()
        ]
        if not eligible:
            return []
        groups = {m.process_group for m in eligible}
        if len(groups) != 1:
            return []
        group = next(iter(groups))
        bounds = [m.sync_timeout for m in eligible if getattr(m, "sync_timeout", None) is not None]
        timeout = min(bounds) if bounds else None
        batches: List[List[Metric]] = [[]]
        size = 0
        for m in eligible:
            batches[-1].append(m)
            # only all-reduced states count: their shapes agree on every rank, so every rank cuts the groups at the
            # same members ('cat' / None / custom states may differ in size per rank)
            size += sum(
                v.numel() * v.element_size()
                for k, v in m.metric_state.items()
                if isinstance(v, Tensor) and m._reductions.get(k) in _ALLREDUCED
            )
            if size >= self._OVERLAP_GROUP_BYTES:
                batches.append([])
                size = 0
        for batch in batches:
            if not batch:
                continue
            pending = PendingSyncMany([m.metric_state for m in batch], [m._reductions for m in batch], group, timeout)
            for i, m in enumerate(batch):
                self._pending_sync[id(m)] = (pending, batch, i)
        eligible_ids = {id(m) for m in eligible}
        if self._groups_checked:
            affected = [getattr(self, n) for cg in self._groups.values() if id(getattr(self, cg[0])) in eligible_ids for n in cg]
        else:
            affected = eligible
        restore: List[Tuple[Metric, bool]] = []
        for m in affected:
            restore.append((m, m._to_sync))
            m._to_sync = False
        return restore

    def _install_pending(self, m: Metric) -> None:
        """Wait for the async sync group holding ``m`` (or its compute-group leader) and install the synced states."""
        pend = getattr(self, "_pending_sync", None)
        if not pend:
            return
        key = id(m)
        if key not in pend and self._groups_checked:
            for cg in self._groups.values():
                names = [n for n in cg if getattr(self, n) is m]
                if names:
                    key = id(getattr(self, cg[0]))
                    break
        entry = pend.get(key)
        if entry is None:
            return
        pending, batch, _ = entry
        synced = pending.wait()
        for bm, new_states in zip(batch, synced):
            pend.pop(id(bm), None)
            bm._cache = bm.metric_state
            for k, v in new_states.items():
                setattr(bm, k, v)
            bm._is_synced = True
        if self._groups_checked:
            self._compute_groups_create_state_ref()

    def _collection_unsync(self, restore: List[Tuple[Metric, bool]]) -> None:
        pend = getattr(self, "_pending_sync", None)
        if pend:  # a member raised before computing: still complete its collectives (every rank issued them)
            for m in [getattr(self, n) for n in self._leaders()]:
                self._install_pending(m)
        if not restore:
            return
        for m, to_sync in restore:
            m._to_sync = to_sync
            if m._is_synced and m._cache is not None:
                m.unsync()
        if self._groups_checked:
            self._compute_groups_create_state_ref()

    def _forward_fused(self, args: Tuple, kwargs: Dict[str, Any]) -> Dict[str, Any]:
        """``forward`` of plan members through the fused update: every eligible member (reduce-state forward) parks
        its global state, the plan updates all of them from one pass over the inputs, and each member computes
        its batch value and merges the global state back (``Metric._fused_forward_begin/_end``)."""
        from torchmetrics_forked_amd.ops.fused import build_fused_plans

        if self._fused_plans is None:
            self._fused_plans = build_fused_plans(self._modules)
        out: Dict[str, Any] = {}
        for plan in self._fused_plans:
            mods = {n: self._modules[n] for n in plan.names if n in self._modules and n not in out}
            mods = {n: m for n, m in mods.items() if m._fused_forward_ok()}
            if len(mods) < 2:
                continue
            ctx = {n: m._fused_forward_begin() for n, m in mods.items()}
            done = set(plan.run(mods, args, kwargs))
            for n, m in mods.items():
                if n not in done:
                    m.update(*args, **m._filter_kwargs(**kwargs))
            for n, m in mods.items():
                out[n] = m._fused_forward_end(ctx[n])
        return out

    def _forward_step_synced(self, args: Tuple, kwargs: Dict[str, Any], skip: Dict[str, Any]) -> Dict[str, Any]:
        """``dist_sync_on_step`` members under DDP: launch every member's batch-state collectives, then compute the
        batch values in order (``Metric._step_sync_begin/_end``) — member i computes while member j's RCCL work runs."""
        from torchmetrics_forked_amd.parallel.sync import distributed_available

        if not distributed_available():
            return {}
        mods = {k: m for k, m in self.items(keep_base=True, copy_state=False) if k not in skip and m._step_sync_ok()}
        if not mods:
            return {}
        # exception-safe: a member whose begin or end raises must not strand the others in batch mode with their
        # global state parked in a ctx (and their launched collectives unwaited) -- every started member is finished
        ctx: Dict[str, Any] = {}
        out: Dict[str, Any] = {}
        try:
            for k, m in mods.items():
                ctx[k] = m._step_sync_begin(args, m._filter_kwargs(**kwargs))
        except BaseException:
            for k in list(ctx):
                try:
                    mods[k]._step_sync_end(ctx.pop(k))
                except Exception:  # noqa: S110 - the first error is the one to report
                    pass
            raise
        err: Optional[BaseException] = None
        for k in list(ctx):
            try:
                out[k] = mods[k]._step_sync_end(ctx.pop(k))
            except BaseException as e:  # finish (restore) the remaining members, then re-raise the first error
                if err is None:
                    err = e
        if err is not None:
            raise err
        return out

    def _compute_and_reduce(self, method_name: str, *args: Any, **kwargs: Any) -> Dict[str, Any]:
        result = {}
        fused = self._forward_fused(args, kwargs) if method_name == "forward" else {}
        if method_name == "forward":
            fused.update(self._forward_step_synced(args, kwargs, fused))
        for k, m in self.items(keep_base=True, copy_state=False):
            if method_name == "compute":
                self._install_pending(m)
                res = m.compute()
            elif method_name == "forward" and k in fused:
                res = fused[k]
            elif method_name == "forward":
                res = m(*args, **m._filter_kwargs(**kwargs))
            else:
                raise ValueError(f"method_name should be either 'compute' or 'forward', but got {method_name}")
            result[k] = res
        _, duplicates = _flatten_dict(result)
        flat: Dict[str, Any] = {}
        for k, m in self.items(keep_base=True, copy_state=False):
            res = result[k]
            if isinstance(res, dict):
                for key, v in res.items():
                    if duplicates:
                        stripped = k.replace(getattr(m, "prefix", "") or "", "").replace(getattr(m, "postfix", "") or "", "")
                        key = f"{stripped}_{key}"
                    if getattr(m, "_from_collection", None) and m.prefix is not None:
                        key = f"{m.prefix}{key}"
                    if getattr(m, "_from_collection", None) and m.postfix is not None:
                        key = f"{key}{m.postfix}"
                    flat[key] = v
            else:
                flat[k] = res
        return {self._set_name(k): v for k, v in flat.items()}

    def reset(self) -> None:
        for m in self.values(copy_state=False):
            m.reset()
        if self._enable_compute_groups and self._groups_checked:
            self._compute_groups_create_state_ref()

    def clone(self, prefix: Optional[str] = None, postfix: Optional[str] = None) -> "MetricCollection":
        mc = deepcopy(self)
        if prefix:
            mc.prefix = self._check_arg(prefix, "prefix")
        if postfix:
            mc.postfix = self._check_arg(postfix, "postfix")
        return mc

    def persistent(self, mode: bool = True) -> None:
        for m in self.values(copy_state=False):
            m.persistent(mode)

    # ------------------------------------------------------------------------------------- membership
    def add_metrics(self, metrics: Union[Metric, Sequence[Metric], Dict[str, Metric]], *additional_metrics: Metric) -> None:
        if isinstance(metrics, Metric):
            metrics = [metrics]
        if isinstance(metrics, Sequence):
            metrics = list(metrics)
            extra: list = []
            for m in additional_metrics:
                (metrics if isinstance(m, Metric) else extra).append(m)
            if extra:
                rank_zero_warn(f"You have passes extra arguments {extra} which are not `Metric` so they will be ignored.")
        elif additional_metrics:
            raise ValueError(
                f"You have passes extra arguments {additional_metrics} which are not compatible"
                f" with first passed dictionary {metrics} so they will be ignored."
            )

        def _absorb(coll: "MetricCollection", key_fn: Any) -> None:
            for k, v in coll.items(keep_base=False):
                v.postfix = coll.postfix
                v.prefix = coll.prefix
                v._from_collection = True
                self[key_fn(k)] = v

        if isinstance(metrics, dict):
            for name in sorted(metrics.keys()):
                metric = metrics[name]
                if not isinstance(metric, (Metric, MetricCollection)):
                    raise ValueError(
                        f"Value {metric} belonging to key {name} is not an instance of"
                        " `torchmetrics.Metric` or `torchmetrics.MetricCollection`"
                    )
                if isinstance(metric, Metric):
                    self[name] = metric
                else:
                    _absorb(metric, lambda k, _n=name: f"{_n}_{k}")
        elif isinstance(metrics, Sequence):
            for metric in metrics:
                if not isinstance(metric, (Metric, MetricCollection)):
                    raise ValueError(
                        f"Input {metric} to `MetricCollection` is not a instance of"
                        " `torchmetrics.Metric` or `torchmetrics.MetricCollection`"
                    )
                if isinstance(metric, Metric):
                    name = metric.__class__.__name__
                    if name in self:
                        raise ValueError(f"Encountered two metrics both named {name}")
                    self[name] = metric
                else:
                    _absorb(metric, lambda k: k)
        else:
            raise ValueError(
                "Unknown input to MetricCollection. Expected, `Metric`, `MetricCollection` or `dict`/`sequence` of the"
                f" previous, but got {metrics}"
            )
        self._groups_checked = False
        self._fused_plans = None
        if self._enable_compute_groups:
            self._init_compute_groups()
        else:
            self._groups = {}

    def _init_compute_groups(self) -> None:
        if isinstance(self._enable_compute_groups, list):
            self._groups = dict(enumerate(self._enable_compute_groups))
            for members in self._groups.values():
                for metric in members:
                    if metric not in self:
                        raise ValueError(
                            f"Input {metric} in `compute_groups` argument does not match a metric in the collection."
                            f" Please make sure that {self._enable_compute_groups} matches {self.keys(keep_base=True)}"
                        )
            self._groups_checked = True
        else:
            self._groups = {i: [str(k)] for i, k in enumerate(self.keys(keep_base=True))}

    @property
    def compute_groups(self) -> Dict[int, List[str]]:
        return self._groups

    def _set_name(self, base: str) -> str:
        name = base if self.prefix is None else self.prefix + base
        return name if self.postfix is None else name + self.postfix

    def _to_renamed_ordered_dict(self) -> OrderedDict:
        return OrderedDict((self._set_name(k), v) for k, v in self._modules.items())

    def __iter__(self) -> Iterator[Hashable]:
        return iter(self.keys())

    def keys(self, keep_base: bool = False) -> Iterable[Hashable]:
        if keep_base:
            return self._modules.keys()
        return self._to_renamed_ordered_dict().keys()

    def items(self, keep_base: bool = False, copy_state: bool = True) -> Iterable[Tuple[str, Metric]]:
        self._compute_groups_create_state_ref(copy_state)
        if keep_base:
            return self._modules.items()
        return self._to_renamed_ordered_dict().items()

    def values(self, copy_state: bool = True) -> Iterable[Metric]:
        self._compute_groups_create_state_ref(copy_state)
        return self._modules.values()

    def __getitem__(self, key: str, copy_state: bool = True) -> Metric:
        self._compute_groups_create_state_ref(copy_state)
        return self._modules[key]

    @staticmethod
    def _check_arg(arg: Optional[str], name: str) -> Optional[str]:
        if arg is None or isinstance(arg, str):
            return arg
        raise ValueError(f"Expected input `{name}` to be a string, but got {type(arg)}")

    def __repr__(self) -> str:
        repr_str = super().__repr__()[:-2]
        if self.prefix:
            repr_str += f",\n  prefix={self.prefix}{',' if self.postfix else ''}"
        if self.postfix:
            repr_str += f"{',' if not self.prefix else ''}\n  postfix={self.postfix}"
        return repr_str + "\n)"

    def set_dtype(self, dst_type: Union[str, torch.dtype]) -> "MetricCollection":
        for m in self.values(copy_state=False):
            m.set_dtype(dst_type)
        return self

    def plot(
        self,
        val: Optional[Union[Dict, Sequence[Dict]]] = None,
        ax: Optional[Union[_AX_TYPE, Sequence[_AX_TYPE]]] = None,
        together: bool = False,
    ) -> Sequence[_PLOT_OUT_TYPE]:
        """Plot every member (one figure each, or all on one axis with ``together=True``)."""
        if not isinstance(together, bool):
            raise ValueError(f"Expected argument `together` to be a boolean, but got {type(together)}")
        if ax is not None:
            if together and not isinstance(ax, _AX_TYPE):
                raise ValueError(f"Expected argument `ax` to be a matplotlib axis object, but got {type(ax)} when `together=True`")
            if not together and not (isinstance(ax, Sequence) and all(isinstance(a, _AX_TYPE) for a in ax) and len(ax) == len(self)):
                raise ValueError(
                    f"Expected argument `ax` to be a sequence of matplotlib axis objects with the same length as the "
                    f"number of metrics in the collection, but got {type(ax)} with len {len(ax)} when `together=False`"
                )
        val = val or self.compute()
        if together:
            return plot_single_or_multi_val(val, ax=ax)
        fig_axs = []
        for i, (k, m) in enumerate(self.items(keep_base=True, copy_state=False)):
            if isinstance(val, dict):
                f, a = m.plot(val[k], ax=ax[i] if ax is not None else ax)
            elif isinstance(val, Sequence):
                f, a = m.plot([v[k] for v in val], ax=ax[i] if ax is not None else ax)
            fig_axs.append((f, a))
        return fig_axs
