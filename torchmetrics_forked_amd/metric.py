"""The ``Metric`` runtime (behavioural contract: reference ``metric.py:50-1198``).

A metric is an ``nn.Module`` whose *states* (registered with :meth:`Metric.add_state`) live on the metric's
device and are merged across processes by the coalesced sync engine (:mod:`..parallel.sync`).

MI355X-first choices that differ from the reference while keeping its observable contract:

* ``sync`` uses one ``all_reduce`` per (op, dtype) bucket for sum/mean/min/max states and a single packed
  all-gather for list/``cat``/``None`` states, instead of barrier + shape-gather + payload-gather per leaf.
  A user supplied ``dist_sync_fn`` still gets the per-leaf protocol.
* ``forward`` on the reduce-state path merges batch state into the global state without re-allocating
  defaults on the host for every step (``_reset_states`` clones device defaults in place).
* Optional ``sync(async_op=True)`` enqueues the coalesced all-reduce buckets on RCCL (``async_op`` work handles)
  and returns immediately, so other GPU work overlaps the xGMI transfer; ``handle.wait()`` installs the states.
"""
import builtins
import functools
import inspect
import os
from abc import ABC, abstractmethod
from contextlib import contextmanager
from copy import deepcopy
from typing import Any, Callable, ClassVar, Dict, Generator, List, Optional, Sequence, Tuple, Union

import torch
from torch import Tensor
from torch.nn import Module

from torchmetrics_forked_amd.parallel.sync import PendingSync, legacy_sync_states, sync_states, sync_states_async, sync_timeout
from torchmetrics_forked_amd.utilities.data import (
    _flatten,
    _squeeze_if_scalar,
    apply_to_collection,
    dim_zero_cat,
    dim_zero_max,
    dim_zero_mean,
    dim_zero_min,
    dim_zero_sum,
)
from torchmetrics_forked_amd.utilities.arena import StateArena
from torchmetrics_forked_amd.utilities.distributed import gather_all_tensors
from torchmetrics_forked_amd.utilities.exceptions import TorchMetricsUserError

# Opt-in tracing: with TMX_PROFILE=1 every update / compute / sync is wrapped in a profiler range
# ("tmx/<Metric>.update", ...), visible in torch.profiler traces and rocprofv3 --marker-trace timelines.
_PROFILE = os.environ.get("TMX_PROFILE", "0") == "1"


def _range(name: str) -> Any:
    if _PROFILE:
        return torch.profiler.record_function(name)
    return _NULL_RANGE


class _NullRange:
    def __enter__(self) -> None:
        return None

    def __exit__(self, *_: Any) -> None:
        return None


_NULL_RANGE = _NullRange()
from torchmetrics_forked_amd.utilities.plot import _AX_TYPE, _PLOT_OUT_TYPE, plot_single_or_multi_val
from torchmetrics_forked_amd.utilities.prints import rank_zero_warn
from torchmetrics_forked_amd.utilities.validation import (
    DeferredChecks,
    enter_forward,
    forward_scope,
    host_checks,
    leave_forward,
    make_sink,
    validation_mode,
)

_PLAIN_ATTR_TYPES = frozenset({Tensor, int, float, bool, str, type(None), tuple, list, dict, StateArena})

_STR_REDUCTIONS = {
    "sum": dim_zero_sum,
    "mean": dim_zero_mean,
    "max": dim_zero_max,
    "min": dim_zero_min,
    "cat": dim_zero_cat,
}
_CONST_ATTRS = frozenset(
    ("higher_is_better", "is_differentiable", "full_state_update", "plot_lower_bound", "plot_upper_bound", "plot_legend_name")
)
_BOOL_KWARGS = ("compute_on_cpu", "dist_sync_on_step", "sync_on_compute", "compute_with_cache", "sharded_compute")


def jit_distributed_available() -> bool:
    return torch.distributed.is_available() and torch.distributed.is_initialized()


class Metric(Module, ABC):
    """Base class of every metric.

    Subclasses register states in ``__init__`` with :meth:`add_state` and implement ``update`` (accumulate a
    batch into the states) and ``compute`` (final value from the states).

    Keyword Args:
        compute_on_cpu: move list states to CPU after each ``update`` (saves device memory).
        dist_sync_on_step: synchronise states on every ``forward`` call.
        process_group: process group used for synchronisation (default: world).
        dist_sync_fn: custom per-tensor gather function (switches to the legacy per-leaf protocol).
        distributed_available_fn: callable deciding whether we run distributed.
        sync_on_compute: synchronise states when ``compute`` is called (default True).
        compute_with_cache: cache ``compute`` output until the next ``update`` (default True).
        sharded_compute: framework extension. Metrics that support state-parallel compute
            reduce-scatter their per-class state across ranks at sync time, compute only their own classes and
            all-gather the small per-class results; others ignore the flag.  Results are identical.
        sync_timeout: framework extension (SURVEY §5 failure detection). Seconds every sync collective may take
            before :class:`~torchmetrics_forked_amd.parallel.sync.SyncTimeoutError` is raised (default: the
            ``TMX_SYNC_TIMEOUT`` environment variable, else unbounded as in the reference).
    """

    __jit_ignored_attributes__: ClassVar[List[str]] = ["device", "_fast_update"]
    __jit_unused_properties__: ClassVar[List[str]] = [
        "is_differentiable",
        "higher_is_better",
        "plot_lower_bound",
        "plot_upper_bound",
        "plot_legend_name",
        "metric_state",
        "_update_called",
    ]
    is_differentiable: Optional[bool] = None
    higher_is_better: Optional[bool] = None
    full_state_update: Optional[bool] = None

    plot_lower_bound: Optional[float] = None
    plot_upper_bound: Optional[float] = None
    plot_legend_name: Optional[str] = None

    def __init__(self, **kwargs: Any) -> None:
        super().__init__()
        torch._C._log_api_usage_once(f"torchmetrics_forked_amd.metric.{self.__class__.__name__}")
        self._device = torch.device("cpu")

        opts = {
            "compute_on_cpu": kwargs.pop("compute_on_cpu", False),
            "dist_sync_on_step": kwargs.pop("dist_sync_on_step", False),
            "sync_on_compute": kwargs.pop("sync_on_compute", True),
            "compute_with_cache": kwargs.pop("compute_with_cache", True),
            "sharded_compute": kwargs.pop("sharded_compute", False),
        }
        for key in _BOOL_KWARGS:
            if not isinstance(opts[key], bool):
                article = "a" if key in ("sync_on_compute", "compute_with_cache", "sharded_compute") else "an"
                raise ValueError(f"Expected keyword argument `{key}` to be {article} `bool` but got {opts[key]}")
            setattr(self, key, opts[key])

        self.process_group = kwargs.pop("process_group", None)
        self.dist_sync_fn = kwargs.pop("dist_sync_fn", None)
        if self.dist_sync_fn is not None and not callable(self.dist_sync_fn):
            raise ValueError(
                f"Expected keyword argument `dist_sync_fn` to be an callable function but got {self.dist_sync_fn}"
            )
        self.distributed_available_fn = kwargs.pop("distributed_available_fn", None) or jit_distributed_available
        self.sync_timeout = kwargs.pop("sync_timeout", None)
        if self.sync_timeout is not None and (isinstance(self.sync_timeout, bool) or not isinstance(self.sync_timeout, (int, float)) or self.sync_timeout <= 0):
            raise ValueError(f"Expected keyword argument `sync_timeout` to be a positive number of seconds but got {self.sync_timeout}")
        if kwargs:
            raise ValueError(f"Unexpected keyword arguments: {', '.join(f'`{k}`' for k in sorted(kwargs))}")

        self._update_signature = inspect.signature(self.update)
        self.update: Callable = self._wrap_update(self.update)  # type: ignore[method-assign]
        self.compute: Callable = self._wrap_compute(self.compute)  # type: ignore[method-assign]
        self._computed: Any = None
        self._forward_cache: Any = None
        self._update_count = 0
        self._to_sync = self.sync_on_compute
        self._should_unsync = True
        self._enable_grad = False
        self._dtype_convert = False

        self._defaults: Dict[str, Union[List, Tensor]] = {}
        self._persistent: Dict[str, bool] = {}
        self._reductions: Dict[str, Union[str, Callable[..., Any], None]] = {}

        self._is_synced = False
        self._cache: Optional[Dict[str, Union[List[Tensor], Tensor]]] = None
        self._deferred: Optional[DeferredChecks] = None

    def _validation_sink(self, t: Tensor) -> Optional[DeferredChecks]:
        """Deferred-validation sink for GPU inputs (flags checked at ``compute``), ``None`` = raise eagerly."""
        mode = validation_mode()
        if mode == "eager" or (mode == "auto" and not t.is_cuda):
            return None
        if self._deferred is None:
            self._deferred = DeferredChecks()
        return self._deferred

    # ------------------------------------------------------------------------------------------------ props
    @property
    def _update_called(self) -> bool:
        rank_zero_warn(
            "This property will be removed in 2.0.0. Use `Metric.updated_called` instead.", DeprecationWarning, stacklevel=2
        )
        return self.update_called

    @property
    def update_called(self) -> bool:
        return self._update_count > 0

    @property
    def update_count(self) -> int:
        return self._update_count

    @property
    def metric_state(self) -> Dict[str, Union[List[Tensor], Tensor]]:
        self._join_side_work()
        return {name: getattr(self, name) for name in self._defaults}

    # ---- deferred state work ---------------------------------------------------------------------------------
    # An update may leave a pending fix-up of this metric's states (CatMetric drops NaN entries once, at the first
    # consumer, instead of synchronising the host per update).  ``_side_event`` holds it; every consumer of the states
    # (compute, sync, reset, state_dict, pickling, device moves, forward) runs it first.
    _side_event: Optional[Any] = None

    def _join_side_work(self) -> None:
        ev = self.__dict__.get("_side_event")
        if ev is not None:
            self.__dict__["_side_event"] = None
            ev()

    @property
    def device(self) -> "torch.device":
        return self._device

    # ----------------------------------------------------------------------------------------------- states
    def add_state(
        self,
        name: str,
        default: Union[list, Tensor],
        dist_reduce_fx: Optional[Union[str, Callable]] = None,
        persistent: bool = False,
    ) -> None:
        """Register a state: a tensor, or an empty list that ``update`` appends tensors to.

        ``dist_reduce_fx`` is one of ``"sum" | "mean" | "max" | "min" | "cat"``, a callable applied to the
        stacked ``(world, ...)`` state, or ``None`` (states are gathered, not reduced).
        """
        if not isinstance(default, (Tensor, list)) or (isinstance(default, list) and default):
            raise ValueError("state variable must be a tensor or any empty list (where you can append tensors)")
        if isinstance(dist_reduce_fx, str) or dist_reduce_fx is None:
            if dist_reduce_fx is not None and dist_reduce_fx not in _STR_REDUCTIONS:
                raise ValueError("`dist_reduce_fx` must be callable or one of ['mean', 'sum', 'cat', 'min', 'max', None]")
            fx = _STR_REDUCTIONS.get(dist_reduce_fx) if dist_reduce_fx is not None else None
        elif callable(dist_reduce_fx):
            fx = dist_reduce_fx
        else:
            raise ValueError("`dist_reduce_fx` must be callable or one of ['mean', 'sum', 'cat', 'min', 'max', None]")
        if isinstance(default, Tensor):
            default = default.contiguous()
        setattr(self, name, default if isinstance(default, Tensor) else StateArena())
        self._defaults[name] = deepcopy(default)
        self._persistent[name] = persistent
        self._reductions[name] = fx
        # an all-zero tensor default (decided here, while it is still a host / freshly built tensor) resets by a fill,
        # not by a device copy of the default: half the memory traffic for large states (a 1000 x 1000 confusion matrix)
        zd = self.__dict__.setdefault("_zero_default", {})
        zd[name] = isinstance(default, Tensor) and default.device.type == "cpu" and default.numel() > 0 and not bool(default.any())

    # ---------------------------------------------------------------------------------------------- forward
    @torch.jit.unused
    def forward(self, *args: Any, **kwargs: Any) -> Any:
        """Accumulate the batch into the global state and return the metric value on this batch alone."""
        enter_forward()  # forward_scope() without the generator context manager (a few us per CPU forward)
        try:
            return self._forward_impl(*args, **kwargs)
        finally:
            leave_forward()

    def _forward_impl(self, *args: Any, **kwargs: Any) -> Any:
        if self._is_synced:
            raise TorchMetricsUserError(
                "The Metric shouldn't be synced when performing ``forward``. HINT: Did you forget to call ``unsync`` ?."
            )
        self._join_side_work()  # pending state work (deferred NaN drops) before states are cached
        if self.dist_sync_on_step and self._step_sync_ok() and self.distributed_available_fn():
            # batch-state collectives launched first, the global update runs beside them (``_step_sync_begin``)
            self._forward_cache = self._step_sync_end(self._step_sync_begin(args, kwargs))
            return self._forward_cache
        full = self.full_state_update or self.full_state_update is None or self.dist_sync_on_step
        if self._deferred is None:
            self._forward_cache = (self._forward_full_state_update if full else self._forward_reduce_state_update)(*args, **kwargs)
            return self._forward_cache
        # the batch value's compute checks (and clears) only the batch's deferred flags; the ones accumulated by
        # earlier update() calls are kept for the user's compute()
        snap = self._deferred.take_for_forward()
        try:
            self._forward_cache = (self._forward_full_state_update if full else self._forward_reduce_state_update)(*args, **kwargs)
        finally:
            self._deferred.give_back(snap)
        return self._forward_cache

    def _enter_batch_mode(self) -> bool:
        d = self.__dict__  # plain attributes: no __setattr__ round trips (a CPU forward is ~20 of them)
        d["_to_sync"] = d["dist_sync_on_step"]
        d["_should_unsync"] = False
        saved = d["compute_on_cpu"]
        d["compute_on_cpu"] = False
        d["_enable_grad"] = True
        return saved

    def _leave_batch_mode(self, saved_compute_on_cpu: bool) -> None:
        d = self.__dict__
        d["_is_synced"] = False
        d["_cache"] = None  # the batch compute's pre-sync states (a batch sync is never unsynced): do not pin them
        d["_should_unsync"] = True
        d["_to_sync"] = d["sync_on_compute"]
        d["_computed"] = None
        d["_enable_grad"] = False
        d["compute_on_cpu"] = saved_compute_on_cpu
        if saved_compute_on_cpu:
            self._move_list_states_to_cpu()

    def _all_tensor_states(self) -> bool:
        """Every state is a tensor (no ``cat`` arena whose views a result could alias); cached per instance."""
        d = self.__dict__
        v = d.get("_tensor_states")
        if v is None:
            v = d["_tensor_states"] = bool(self._defaults) and all(isinstance(x, Tensor) for x in self._defaults.values())
        return v

    def _sum_forward_names(self) -> Optional[Tuple[str, ...]]:
        """State names when every state is a tensor merged by sum and neither ``reset`` nor ``_reduce_states`` is
        overridden: ``forward`` may then build the batch state from the defaults and merge with one ``_foreach_add``
        (cached per instance; ``None`` otherwise)."""
        d = self.__dict__
        cached = d.get("_sum_fwd")
        if cached is not None:
            return cached or None
        cls = type(self)
        ok = (
            cls.reset is Metric.reset and cls._reduce_states is Metric._reduce_states and bool(self._defaults)
            and all(isinstance(v, Tensor) for v in self._defaults.values())
            and all(self._reductions[n] is dim_zero_sum for n in self._defaults)
        )
        names = tuple(self._defaults) if ok else ()
        d["_sum_fwd"] = names
        d["_sum_fwd_defaults"] = [self._defaults[n] for n in names]
        d["_sum_fwd_zero"] = all(not bool(self._defaults[n].any()) for n in names)
        d["_sum_fwd_scratch"] = None
        return names or None

    def _forward_full_state_update(self, *args: Any, **kwargs: Any) -> Any:
        """Two ``update`` calls: one into the global state, one into a fresh state for the batch value."""
        self.update(*args, **kwargs)
        count = self._update_count
        saved = self._enter_batch_mode()
        snapshot = self.metric_state
        self.reset()
        self.update(*args, **kwargs)
        batch_val = self.compute()
        for name, val in snapshot.items():
            setattr(self, name, val)
        self._update_count = count
        self._leave_batch_mode(saved)
        return batch_val

    def _forward_reduce_state_update(self, *args: Any, **kwargs: Any) -> Any:
        """One ``update`` into a fresh state; the batch state is then merged into the global state."""
        names = self._sum_forward_names()
        d = self.__dict__
        if names is not None and d.get("_side_event") is None:
            # sum-merged tensor states (stat scores, confusion matrices, regression sums ...): the reset below is
            # Metric.reset restricted to what a batch needs, the merge one fused add -- same states, same values
            try:
                glob = [d[n] for n in names]
            except KeyError:  # a state not held as a plain attribute: the generic path
                glob = None
        else:
            glob = None
        if glob is not None:
            defaults = d["_sum_fwd_defaults"]
            scratch = d.get("_sum_fwd_scratch")
            if scratch is not None and scratch[0].device == glob[0].device:
                fresh = scratch  # the previous forward's batch states, unaliased: zeroed in one call (zero defaults)
                torch._foreach_zero_(fresh)
            elif defaults[0].device == glob[0].device:  # states and defaults move together (_apply)
                fresh = torch._foreach_add(defaults, 0)  # one call: a fresh copy of every default
            else:
                fresh = [dv.detach().clone().to(g.device) for dv, g in zip(defaults, glob)]
            for n, f in zip(names, fresh):
                d[n] = f
            count = d["_update_count"]
            d["_update_count"] = 0
            d["_forward_cache"] = None
            d["_computed"] = None
            d["_cache"] = None
            d["_is_synced"] = False
            if self._deferred is not None:
                self._deferred.clear()
            saved = self._enter_batch_mode()
            self.update(*args, **kwargs)
            batch_val = self.compute()
            d["_update_count"] = count + 1
            batch = [d[n] for n in names]  # (an update may have rebound a state rather than added into it)
            with torch.no_grad():
                # out of place, as the reference's ``global + local`` (metric.py:_reduce_states): a compute group's
                # members share the leader's state tensors, so an in-place merge would add each batch once per member;
                # the new tensors also take the reference's type promotion (int64 state + float batch -> float)
                glob = torch._foreach_add(glob, batch)
            for n, g in zip(names, glob):
                d[n] = g
            # keep the batch states for the next forward when they are zero-defaulted and the batch value does not
            # alias them (a confusion matrix's compute returns its state)
            if d["_sum_fwd_zero"]:
                # the storage addresses of a reused scratch are known from the previous forward
                ptrs = d.get("_sum_fwd_ptrs") if fresh is scratch and all(a is b for a, b in zip(batch, fresh)) else None
                if ptrs is None:
                    ptrs = {t.untyped_storage().data_ptr() for t in batch}
                d["_sum_fwd_ptrs"] = ptrs
                d["_sum_fwd_scratch"] = None if _aliases(batch_val, ptrs) else batch
            else:
                d["_sum_fwd_scratch"] = None
            self._leave_batch_mode(saved)
            return batch_val
        snapshot = self.metric_state
        count = self._update_count
        self.reset()
        saved = self._enter_batch_mode()
        self.update(*args, **kwargs)
        batch_val = self.compute()
        self._update_count = count + 1
        with torch.no_grad():
            self._reduce_states(snapshot)
        self._leave_batch_mode(saved)
        return batch_val

    # ---- overlapped dist_sync_on_step (Metric.forward and MetricCollection.forward) ------------------------------
    # The reference syncs and computes each batch value in turn (``metric.py:273-305``): global update, batch update,
    # then a blocking gather inside compute.  Here the batch update runs first and its collectives are launched at once
    # (``sync(async_op=True)``: coalesced buckets enqueued on RCCL's stream); the global-state update then runs while
    # they are in flight (it touches other tensors), and only the batch compute waits for them.  A collection launches
    # every member's collectives before computing any batch value, so member i computes while member j's sync runs.
    def _step_sync_ok(self) -> bool:
        from torchmetrics_forked_amd.utilities.distributed import gather_all_tensors

        return (
            self.dist_sync_on_step and not self._is_synced and type(self)._sync_dist is Metric._sync_dist
            and (self.dist_sync_fn is None or self.dist_sync_fn is gather_all_tensors)
        )

    def _step_sync_begin(self, args: Tuple, kwargs: Dict[str, Any]) -> Tuple[Any, ...]:
        """First half of ``forward`` with ``dist_sync_on_step``: fresh batch state, batch update, batch-state
        collectives launched, then the global update beside them.  On an exception the global state is restored
        (and launched collectives completed, since every rank issued them) before it propagates."""
        self._join_side_work()
        snap_def = None
        if self._deferred is not None:
            snap_def = self._deferred.take_for_forward()
        count = self._update_count
        glob = self.metric_state
        saved = self._enter_batch_mode()
        handle = None
        try:
            self.reset()
            self.update(*args, **kwargs)
            handle = self.sync(dist_sync_fn=self.dist_sync_fn, async_op=True)
            batch = self.metric_state
            for name, val in glob.items():
                setattr(self, name, val)
            self._update_count = count
            self._enable_grad, self.compute_on_cpu = False, saved  # the global update as a plain update() call
            try:
                self.update(*args, **kwargs)
            finally:
                self._enable_grad, self.compute_on_cpu = True, False
            glob, count = self.metric_state, self._update_count
            for name, val in batch.items():
                setattr(self, name, val)
            self._update_count = 1
        except BaseException:
            if handle is not None:
                handle.wait()
            self._step_sync_restore(snap_def, count, saved, glob)
            raise
        return snap_def, count, saved, glob, handle

    def _step_sync_restore(self, snap_def: Any, count: int, saved: bool, glob: Dict[str, Any]) -> None:
        for name, val in glob.items():
            setattr(self, name, val)
        self._update_count = count
        self._cache = None
        self._leave_batch_mode(saved)
        if snap_def is not None:
            self._deferred.give_back(snap_def)

    def _step_sync_end(self, ctx: Tuple[Any, ...]) -> Any:
        """Second half: wait for this metric's collectives, compute the synced batch value, restore the global state."""
        snap_def, count, saved, glob, handle = ctx
        try:
            if handle is not None:
                handle.wait()
            self._to_sync = False  # already synced (or not distributed)
            batch_val = self.compute()
        finally:
            self._step_sync_restore(snap_def, count, saved, glob)
        self._forward_cache = batch_val
        return batch_val

    # ---- split reduce-state forward, used by MetricCollection to run one fused update for several members ----
    def _fused_forward_ok(self) -> bool:
        full = self.full_state_update or self.full_state_update is None or self.dist_sync_on_step
        return not full and not self._is_synced

    def _fused_forward_begin(self) -> Tuple[Any, ...]:
        """First half of ``_forward_reduce_state_update``: park the global state (and deferred flags), start a
        fresh batch state; the caller then updates this metric (possibly through a fused collection kernel)."""
        self._join_side_work()
        snap_def = None
        if self._deferred is not None:
            snap_def = self._deferred.take_for_forward()
        snapshot = self.metric_state
        count = self._update_count
        self.reset()
        saved = self._enter_batch_mode()
        return snapshot, count, saved, snap_def

    def _fused_forward_end(self, ctx: Tuple[Any, ...]) -> Any:
        """Second half: batch value from the batch state, then merge the parked global state back in."""
        snapshot, count, saved, snap_def = ctx
        try:
            batch_val = self.compute()
            self._update_count = count + 1
            with torch.no_grad():
                self._reduce_states(snapshot)
            self._leave_batch_mode(saved)
        finally:
            if snap_def is not None:
                self._deferred.give_back(snap_def)
        self._forward_cache = batch_val
        return batch_val

    def _reduce_states(self, incoming_state: Dict[str, Any]) -> None:
        """Merge ``incoming_state`` (global) with the current (batch) state according to each reduction."""
        for name in self._defaults:
            local = getattr(self, name)
            glob = incoming_state[name]
            fx = self._reductions[name]
            if fx is dim_zero_sum:
                merged = glob + local
            elif fx is dim_zero_mean:
                merged = ((self._update_count - 1) * glob + local).float() / self._update_count
            elif fx is dim_zero_max:
                merged = torch.max(glob, local)
            elif fx is dim_zero_min:
                merged = torch.min(glob, local)
            elif fx is dim_zero_cat:
                if isinstance(glob, Tensor) and isinstance(local, Tensor):
                    merged = torch.cat([glob, local])
                else:
                    merged = (StateArena.adopt(glob) if isinstance(glob, StateArena) else StateArena(glob)) if isinstance(glob, list) else glob
                    if isinstance(merged, list):
                        merged.extend(local)
                    else:
                        merged = merged + local
            elif fx is None and isinstance(glob, Tensor):
                merged = torch.stack([glob, local])
            elif fx is None and isinstance(glob, list):
                merged = _flatten([glob, local])
            elif callable(fx):
                merged = fx(torch.stack([glob, local]))
            else:
                raise TypeError(f"Unsupported reduce_fn: {fx}")
            setattr(self, name, merged)

    # ------------------------------------------------------------------------------------------------- sync
    def _sync_dist(self, dist_sync_fn: Optional[Callable] = None, process_group: Optional[Any] = None) -> None:
        states = self.metric_state
        group = process_group or self.process_group
        if dist_sync_fn is None or dist_sync_fn is gather_all_tensors:
            synced = sync_states(states, self._reductions, group=group)
        else:
            synced = legacy_sync_states(states, self._reductions, dist_sync_fn, group=group)
        for name, val in synced.items():
            setattr(self, name, val)

    def _wrap_update(self, update: Callable) -> Callable:
        def run(args: Tuple, kwargs: Dict[str, Any]) -> None:
            try:
                self._check_state_devices(args, kwargs)
                update(*args, **kwargs)
            except RuntimeError as err:
                if "Expected all tensors to be on" in str(err):
                    raise RuntimeError(
                        "Encountered different devices in metric calculation (see stacktrace for details)."
                        " This could be due to the metric class not being on the same device as input."
                        f" Instead of `metric={self.__class__.__name__}(...)` try to do"
                        f" `metric={self.__class__.__name__}(...).to(device)` where"
                        " device corresponds to the device of the input."
                    ) from err
                raise err

        @functools.wraps(update)
        def wrapped_func(*args: Any, **kwargs: Any) -> None:
            d = self.__dict__
            d["_computed"] = None  # plain attributes: no nn.Module __setattr__ round trip on the hot path
            d["_update_count"] += 1
            # the grad-mode context only when the mode actually changes (~2 us per update otherwise)
            if torch.is_grad_enabled() != self._enable_grad:
                with torch.set_grad_enabled(self._enable_grad), _range(f"tmx/{self.__class__.__name__}.update"):
                    run(args, kwargs)
            elif _PROFILE:
                with _range(f"tmx/{self.__class__.__name__}.update"):
                    run(args, kwargs)
            else:
                run(args, kwargs)
            if self.compute_on_cpu:
                self._move_list_states_to_cpu()

        return wrapped_func

    def _check_state_devices(self, args: Tuple, kwargs: Dict[str, Any]) -> None:
        """GPU inputs with a tensor state on another device: raise torch's device error (re-worded by the caller, as in
        the reference) *before* any native kernel runs — a HIP kernel handed a host or other-device state pointer would
        fault the GPU instead of raising.  List states and empty placeholders are created on the input device."""
        dev = None
        for a in args:
            if isinstance(a, Tensor) and a.is_cuda:
                dev = a.device
                break
        if dev is None:
            for a in kwargs.values():
                if isinstance(a, Tensor) and a.is_cuda:
                    dev = a.device
                    break
        if dev is None:
            return
        for name in self._defaults:
            v = getattr(self, name, None)
            if isinstance(v, Tensor) and v.numel() > 0 and v.device != dev and not self._state_device_adapts(name):
                raise RuntimeError(f"Expected all tensors to be on the same device, but found at least two devices, {dev} and {v.device}!")

    def _state_device_adapts(self, name: str) -> bool:
        """States a metric's update moves to the input device itself (override per metric)."""
        return False

    def _move_list_states_to_cpu(self) -> None:
        for name in self._defaults:
            val = getattr(self, name)
            if isinstance(val, Sequence):
                setattr(self, name, [v.to("cpu") if isinstance(v, Tensor) else v for v in val])

    def sync(
        self,
        dist_sync_fn: Optional[Callable] = None,
        process_group: Optional[Any] = None,
        should_sync: bool = True,
        distributed_available: Optional[Callable] = None,
        async_op: bool = False,
    ) -> Optional["_MetricPendingSync"]:
        """Replace local states by their cross-process reduction (local copies are cached for ``unsync``).

        With ``async_op=True`` the all-reduce buckets are only enqueued on RCCL and a handle is returned; the
        caller overlaps other GPU work (e.g. the next step's updates of *other* metrics) and calls
        ``handle.wait()``, which installs the synced states exactly like the blocking path.  States must not be
        updated between the two calls."""
        if self._is_synced and should_sync:
            raise TorchMetricsUserError("The Metric has already been synced.")
        if not should_sync:
            return _MetricPendingSync(self, None) if async_op else None
        if distributed_available is None and self.distributed_available_fn is not None:
            distributed_available = self.distributed_available_fn
        is_distributed = distributed_available() if callable(distributed_available) else None
        if not is_distributed:
            return _MetricPendingSync(self, None) if async_op else None
        if async_op:
            if dist_sync_fn is not None and dist_sync_fn is not gather_all_tensors:
                raise TorchMetricsUserError("`async_op=True` uses the coalesced sync engine; a custom `dist_sync_fn` is not supported.")
            pending = sync_states_async(
                self.metric_state, self._reductions, group=process_group or self.process_group,
                timeout=getattr(self, "sync_timeout", None),
            )
            return _MetricPendingSync(self, pending)
        self._cache = self.metric_state
        with _range(f"tmx/{self.__class__.__name__}.sync"), sync_timeout(getattr(self, "sync_timeout", None)):
            self._sync_dist(dist_sync_fn, process_group=process_group)
        self._is_synced = True
        return None

    def unsync(self, should_unsync: bool = True) -> None:
        """Restore the local (pre-sync) states."""
        if not should_unsync:
            return
        if not self._is_synced:
            raise TorchMetricsUserError("The Metric has already been un-synced.")
        if self._cache is None:
            raise TorchMetricsUserError("The internal cache should exist to unsync the Metric.")
        for name, val in self._cache.items():
            setattr(self, name, val)
        self._is_synced = False
        self._cache = None

    def _finish_async_sync(self, pending: PendingSync) -> None:
        if self._is_synced:
            raise TorchMetricsUserError("The Metric has already been synced.")
        local = self.metric_state
        for name, val in pending.wait().items():
            setattr(self, name, val)
        self._cache = local
        self._is_synced = True

    @contextmanager
    def sync_context(
        self,
        dist_sync_fn: Optional[Callable] = None,
        process_group: Optional[Any] = None,
        should_sync: bool = True,
        should_unsync: bool = True,
        distributed_available: Optional[Callable] = None,
    ) -> Generator:
        """Context manager: synced states inside, local states restored on exit (if we synced)."""
        self.sync(
            dist_sync_fn=dist_sync_fn,
            process_group=process_group,
            should_sync=should_sync,
            distributed_available=distributed_available,
        )
        yield
        self.unsync(should_unsync=self._is_synced and should_unsync)

    def _wrap_compute(self, compute: Callable) -> Callable:
        @functools.wraps(compute)
        def wrapped_func(*args: Any, **kwargs: Any) -> Any:
            if self._update_count == 0:
                rank_zero_warn(
                    f"The ``compute`` method of metric {self.__class__.__name__}"
                    " was called before the ``update`` method which may lead to errors,"
                    " as metric states have not yet been updated.",
                    UserWarning,
                )
            d = self.__dict__
            if d["_computed"] is not None:
                return d["_computed"]
            self._join_side_work()
            if not d["_to_sync"] and d["_deferred"] is None and d["_device"].type == "cpu" and not _PROFILE:
                # host metric, no collective, no device flags: nothing for a host-check block to batch (a check
                # registered by compute reads its CPU flags at once) -- the wrapper's context managers are skipped
                value = compute(*args, **kwargs)
                if type(value) is Tensor:
                    if value.ndim and value.numel() == 1:
                        value = value.squeeze()
                else:
                    value = _squeeze_if_scalar(value)
                if not self._all_tensor_states():
                    value = self._unalias(value)
                if self.compute_with_cache:
                    d["_computed"] = value
                return value
            # every host-side consequence of device flags (deferred input checks, degenerate-class warnings, ...)
            # is read once, when the outermost compute (or MetricCollection.compute) ends
            with host_checks() as batch:
                if self._deferred is not None:
                    self._deferred.check()
                if _PROFILE or d["_is_synced"] or (d["_to_sync"] and self._distributed_on()):
                    with _range(f"tmx/{self.__class__.__name__}.compute"), self.sync_context(
                        dist_sync_fn=self.dist_sync_fn, should_sync=self._to_sync, should_unsync=self._should_unsync
                    ):
                        value = self._unalias(_squeeze_if_scalar(compute(*args, **kwargs)))
                else:  # nothing to sync or unsync (sync_context would return at once): no generator context per compute
                    value = self._unalias(_squeeze_if_scalar(compute(*args, **kwargs)))
                if self.compute_with_cache:
                    self._computed = value
                    batch.on_error(self._drop_computed)
            return value

        return wrapped_func

    def _distributed_on(self) -> bool:
        """``sync``'s own test (``distributed_available_fn``, no override): would a sync reach a collective?"""
        fn = self.distributed_available_fn
        return bool(fn()) if callable(fn) else False

    def _drop_computed(self) -> None:
        self._computed = None

    def _unalias(self, value: Any) -> Any:
        """Copy result tensors that are views of a ``cat`` state's arena buffer (``utilities/arena.py``): the reference's
        ``dim_zero_cat`` returns a fresh tensor, so in-place edits of a result must not reach the accumulated state."""
        arenas = [v for v in (getattr(self, n, None) for n in self._defaults) if isinstance(v, StateArena) and v._buf is not None]
        if not arenas:
            return value

        def fix(x: Any) -> Any:
            if isinstance(x, Tensor):
                return x.clone() if any(a.owns(x) for a in arenas) else x
            if isinstance(x, dict):
                return {k: fix(v) for k, v in x.items()}
            if isinstance(x, (list, tuple)):
                return type(x)(fix(v) for v in x) if not hasattr(x, "_fields") else type(x)(*(fix(v) for v in x))
            return x

        return fix(value)

    @abstractmethod
    def update(self, *_: Any, **__: Any) -> None:
        """Accumulate a batch into the metric states."""

    @abstractmethod
    def compute(self) -> Any:
        """Compute the final metric value from the (synchronised) states."""

    # ------------------------------------------------------------------------------------------------ misc
    def plot(self, *_: Any, **__: Any) -> Any:
        raise NotImplementedError

    def _plot(self, val: Any = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:
        val = val if val is not None else self.compute()
        return plot_single_or_multi_val(
            val,
            ax=ax,
            higher_is_better=self.higher_is_better,
            name=self.__class__.__name__,
            lower_bound=self.plot_lower_bound,
            upper_bound=self.plot_upper_bound,
            legend_name=self.plot_legend_name,
        )

    def reset(self) -> None:
        """Restore every state to its default (on the state's current device)."""
        self._join_side_work()
        self._update_count = 0
        self._forward_cache = None
        self._computed = None
        zero = self.__dict__.get("_zero_default", {})
        for name, default in self._defaults.items():
            if isinstance(default, Tensor):
                current = getattr(self, name)
                dev = current.device if isinstance(current, Tensor) else default.device
                if zero.get(name):
                    setattr(self, name, torch.zeros(default.shape, dtype=default.dtype, device=dev))
                else:
                    setattr(self, name, default.detach().clone().to(dev))
            else:
                setattr(self, name, StateArena())
        self._cache = None
        self._is_synced = False
        if self._deferred is not None:
            self._deferred.clear()

    def clone(self) -> "Metric":
        return deepcopy(self)

    def __getstate__(self) -> Dict[str, Any]:
        self._join_side_work()
        return {k: v for k, v in self.__dict__.items() if k not in ("update", "compute", "_update_signature", "_hist_spare", "_batch_bufs", "_batch_sink", "_batch_view", "_fast_update", "_sum_fwd", "_sum_fwd_defaults", "_sum_fwd_scratch", "_sum_fwd_ptrs", "_tensor_states", "_owned_buf", "_lanes")}

    def __setstate__(self, state: Dict[str, Any]) -> None:
        self.__dict__.update(state)
        self._update_signature = inspect.signature(self.update)
        self.update: Callable = self._wrap_update(self.update)  # type: ignore[method-assign]
        self.compute: Callable = self._wrap_compute(self.compute)  # type: ignore[method-assign]

    def __setattr__(self, name: str, value: Any) -> None:
        if name in _CONST_ATTRS:
            raise RuntimeError(f"Can't change const `{name}`.")
        # Fast path for rebinding an existing plain attribute (states, counters, flags) to a plain value: nn.Module's
        # __setattr__ would only reach object.__setattr__ after its Parameter / Module / buffer checks (~8 us per call,
        # dozens of calls per forward).  Parameters, modules and buffers live in their own dicts, never in __dict__, and
        # the exact-type test keeps Parameter (a Tensor subclass) and every Module on the full path.
        if type(value) in _PLAIN_ATTR_TYPES and name in self.__dict__:
            object.__setattr__(self, name, value)
            return
        super().__setattr__(name, value)

    # dtype casts are no-ops unless routed through set_dtype (reference metric.py:729-760)
    def type(self, dst_type: Union[str, torch.dtype]) -> "Metric":  # noqa: A003
        return self

    def float(self) -> "Metric":  # noqa: A003
        return self

    def double(self) -> "Metric":
        return self

    def half(self) -> "Metric":
        return self

    def set_dtype(self, dst_type: Union[str, torch.dtype]) -> "Metric":
        """Cast every floating state (and default) to ``dst_type``."""
        self._dtype_convert = True
        out = super().type(dst_type)
        out._dtype_convert = False
        return out

    def _apply(self, fn: Callable, exclude_state: Sequence[str] = "") -> Module:
        self._join_side_work()
        for k in ("_sum_fwd", "_sum_fwd_defaults", "_sum_fwd_scratch", "_sum_fwd_ptrs"):  # forward's caches follow the new device / dtype
            self.__dict__.pop(k, None)
        this = super()._apply(fn)
        fs = str(fn)
        is_cast = any(f in fs for f in ("Module.type", "Module.half", "Module.float", "Module.double", "Module.bfloat16"))
        if not self._dtype_convert and is_cast:
            return this
        for key, value in this._defaults.items():
            if key in exclude_state:
                continue
            if isinstance(value, Tensor):
                this._defaults[key] = fn(value)
            elif isinstance(value, Sequence):
                this._defaults[key] = [fn(v) if isinstance(v, Tensor) else v for v in value]
            current = getattr(this, key)
            if isinstance(current, Tensor):
                setattr(this, key, fn(current))
            elif isinstance(current, Sequence):  # non-tensor items (segm RLE tuples) are device independent
                items = (fn(v) if isinstance(v, Tensor) else v for v in current)
                setattr(this, key, StateArena(items) if isinstance(current, StateArena) else list(items))
            else:
                raise TypeError(
                    f"Expected metric state to be either a Tensor or a list of Tensor, but encountered {current}"
                )
        self._device = fn(torch.zeros(1, device=self.device)).device
        if this._computed is not None:
            this._computed = apply_to_collection(this._computed, Tensor, fn)
        if this._forward_cache is not None:
            this._forward_cache = apply_to_collection(this._forward_cache, Tensor, fn)
        return this

    def persistent(self, mode: bool = False) -> None:
        for key in self._persistent:
            self._persistent[key] = mode

    def state_dict(  # type: ignore[override]
        self, destination: Optional[Dict[str, Any]] = None, prefix: str = "", keep_vars: bool = False
    ) -> Dict[str, Any]:
        self._join_side_work()
        destination = super().state_dict(destination=destination, prefix=prefix, keep_vars=keep_vars)  # type: ignore
        for key in self._defaults:
            if not self._persistent[key]:
                continue
            val = getattr(self, key)
            if not keep_vars:
                if isinstance(val, Tensor):
                    val = val.detach()
                elif isinstance(val, StateArena):  # one storage per item, as the reference's lists
                    destination[prefix + key] = val.compact_items()
                    continue
                elif isinstance(val, list):
                    val = [v.detach() if isinstance(v, Tensor) else v for v in val]
            destination[prefix + key] = deepcopy(val)
        return destination

    def _load_from_state_dict(
        self,
        state_dict: dict,
        prefix: str,
        local_metadata: dict,
        strict: bool,
        missing_keys: List[str],
        unexpected_keys: List[str],
        error_msgs: List[str],
    ) -> None:
        self._join_side_work()  # pending state work lands in the states being replaced, not in the loaded ones
        for key in self._defaults:
            name = prefix + key
            if name in state_dict:
                setattr(self, key, state_dict.pop(name))
        super()._load_from_state_dict(state_dict, prefix, local_metadata, True, missing_keys, unexpected_keys, error_msgs)

    def _filter_kwargs(self, **kwargs: Any) -> Dict[str, Any]:
        """Keep only kwargs accepted by ``update`` (all of them if it takes ``**kwargs``)."""
        params = self._update_signature.parameters
        var_kinds = (inspect.Parameter.VAR_POSITIONAL, inspect.Parameter.VAR_KEYWORD)
        has_var_kw = any(p.kind == inspect.Parameter.VAR_KEYWORD for p in params.values())
        if has_var_kw:
            return kwargs
        return {k: v for k, v in kwargs.items() if k in params and params[k].kind not in var_kinds}

    def __hash__(self) -> int:
        vals: List[Any] = [self.__class__.__name__, id(self)]
        for key in self._defaults:
            val = getattr(self, key)
            if hasattr(val, "__iter__") and not isinstance(val, Tensor):
                vals.extend(val)
            else:
                vals.append(val)
        return hash(tuple(vals))

    # ------------------------------------------------------------------------------------- operator algebra
    def __add__(self, other: Any) -> "CompositionalMetric":
        return CompositionalMetric(torch.add, self, other)

    def __and__(self, other: Any) -> "CompositionalMetric":
        return CompositionalMetric(torch.bitwise_and, self, other)

    def __eq__(self, other: Any) -> "CompositionalMetric":  # type: ignore[override]
        return CompositionalMetric(torch.eq, self, other)

    def __floordiv__(self, other: Any) -> "CompositionalMetric":
        return CompositionalMetric(torch.floor_divide, self, other)

    def __ge__(self, other: Any) -> "CompositionalMetric":
        return CompositionalMetric(torch.ge, self, other)

    def __gt__(self, other: Any) -> "CompositionalMetric":
        return CompositionalMetric(torch.gt, self, other)

    def __le__(self, other: Any) -> "CompositionalMetric":
        return CompositionalMetric(torch.le, self, other)

    def __lt__(self, other: Any) -> "CompositionalMetric":
        return CompositionalMetric(torch.lt, self, other)

    def __matmul__(self, other: Any) -> "CompositionalMetric":
        return CompositionalMetric(torch.matmul, self, other)

    def __mod__(self, other: Any) -> "CompositionalMetric":
        return CompositionalMetric(torch.fmod, self, other)

    def __mul__(self, other: Any) -> "CompositionalMetric":
        return CompositionalMetric(torch.mul, self, other)

    def __ne__(self, other: Any) -> "CompositionalMetric":  # type: ignore[override]
        return CompositionalMetric(torch.ne, self, other)

    def __or__(self, other: Any) -> "CompositionalMetric":
        return CompositionalMetric(torch.bitwise_or, self, other)

    def __pow__(self, other: Any) -> "CompositionalMetric":
        return CompositionalMetric(torch.pow, self, other)

    def __radd__(self, other: Any) -> "CompositionalMetric":
        return CompositionalMetric(torch.add, other, self)

    def __rand__(self, other: Any) -> "CompositionalMetric":
        return CompositionalMetric(torch.bitwise_and, self, other)

    def __rfloordiv__(self, other: Any) -> "CompositionalMetric":
        return CompositionalMetric(torch.floor_divide, other, self)

    def __rmatmul__(self, other: Any) -> "CompositionalMetric":
        return CompositionalMetric(torch.matmul, other, self)

    def __rmod__(self, other: Any) -> "CompositionalMetric":
        return CompositionalMetric(torch.fmod, other, self)

    def __rmul__(self, other: Any) -> "CompositionalMetric":
        return CompositionalMetric(torch.mul, other, self)

    def __ror__(self, other: Any) -> "CompositionalMetric":
        return CompositionalMetric(torch.bitwise_or, other, self)

    def __rpow__(self, other: Any) -> "CompositionalMetric":
        return CompositionalMetric(torch.pow, other, self)

    def __rsub__(self, other: Any) -> "CompositionalMetric":
        return CompositionalMetric(torch.sub, other, self)

    def __rtruediv__(self, other: Any) -> "CompositionalMetric":
        return CompositionalMetric(torch.true_divide, other, self)

    def __rxor__(self, other: Any) -> "CompositionalMetric":
        return CompositionalMetric(torch.bitwise_xor, other, self)

    def __sub__(self, other: Any) -> "CompositionalMetric":
        return CompositionalMetric(torch.sub, self, other)

    def __truediv__(self, other: Any) -> "CompositionalMetric":
        return CompositionalMetric(torch.true_divide, self, other)

    def __xor__(self, other: Any) -> "CompositionalMetric":
        return CompositionalMetric(torch.bitwise_xor, self, other)

    def __abs__(self) -> "CompositionalMetric":
        return CompositionalMetric(torch.abs, self, None)

    def __inv__(self) -> "CompositionalMetric":
        return CompositionalMetric(torch.bitwise_not, self, None)

    def __invert__(self) -> "CompositionalMetric":
        return self.__inv__()

    def __neg__(self) -> "CompositionalMetric":
        return CompositionalMetric(_neg, self, None)

    def __pos__(self) -> "CompositionalMetric":
        return CompositionalMetric(torch.abs, self, None)

    def __getitem__(self, idx: int) -> "CompositionalMetric":
        return CompositionalMetric(lambda x: x[idx], self, None)

    def __getnewargs__(self) -> Tuple:
        return (Metric.__str__(self),)

    __iter__ = None


def _neg(x: Tensor) -> Tensor:
    return -torch.abs(x)


class CompositionalMetric(Metric):
    """``op(metric_a.compute(), metric_b.compute())``; update/forward/reset are forwarded to the operands."""

    def __init__(self, operator: Callable, metric_a: Union[Metric, builtins.float, Tensor], metric_b: Union[Metric, builtins.float, Tensor, None]) -> None:
        super().__init__()
        self.op = operator
        if isinstance(metric_a, Tensor):
            self.register_buffer("metric_a", metric_a, persistent=False)
        else:
            self.metric_a = metric_a
        if isinstance(metric_b, Tensor):
            self.register_buffer("metric_b", metric_b, persistent=False)
        else:
            self.metric_b = metric_b

    def _sync_dist(self, dist_sync_fn: Optional[Callable] = None, process_group: Optional[Any] = None) -> None:
        """Operands synchronise themselves."""

    def update(self, *args: Any, **kwargs: Any) -> None:
        if isinstance(self.metric_a, Metric):
            self.metric_a.update(*args, **self.metric_a._filter_kwargs(**kwargs))
        if isinstance(self.metric_b, Metric):
            self.metric_b.update(*args, **self.metric_b._filter_kwargs(**kwargs))

    def compute(self) -> Any:
        val_a = self.metric_a.compute() if isinstance(self.metric_a, Metric) else self.metric_a
        val_b = self.metric_b.compute() if isinstance(self.metric_b, Metric) else self.metric_b
        return self.op(val_a) if val_b is None else self.op(val_a, val_b)

    @torch.jit.unused
    def forward(self, *args: Any, **kwargs: Any) -> Any:
        val_a = self.metric_a(*args, **self.metric_a._filter_kwargs(**kwargs)) if isinstance(self.metric_a, Metric) else self.metric_a
        val_b = self.metric_b(*args, **self.metric_b._filter_kwargs(**kwargs)) if isinstance(self.metric_b, Metric) else self.metric_b
        if val_a is None:
            self._forward_cache = None
            return self._forward_cache
        if val_b is None:
            if isinstance(self.metric_b, Metric):
                self._forward_cache = None
                return self._forward_cache
            self._forward_cache = self.op(val_a)
            return self._forward_cache
        self._forward_cache = self.op(val_a, val_b)
        return self._forward_cache

    def reset(self) -> None:
        if isinstance(self.metric_a, Metric):
            self.metric_a.reset()
        if isinstance(self.metric_b, Metric):
            self.metric_b.reset()

    def persistent(self, mode: bool = False) -> None:
        if isinstance(self.metric_a, Metric):
            self.metric_a.persistent(mode=mode)
        if isinstance(self.metric_b, Metric):
            self.metric_b.persistent(mode=mode)

    def __repr__(self) -> str:
        _op_metrics = f"(\n  {self.op.__name__}(\n    {self.metric_a!r},\n    {self.metric_b!r}\n  )\n)"
        return self.__class__.__name__ + _op_metrics

    def _wrap_compute(self, compute: Callable) -> Callable:
        return compute


def _aliases(value: Any, ptrs: Any) -> bool:
    """True if any tensor in ``value`` (a tensor, or a flat dict / tuple / list of them) shares storage with one of
    the storages at ``ptrs`` (storage data pointers; a list of tensors is converted)."""
    if isinstance(ptrs, list):
        ptrs = {t.untyped_storage().data_ptr() for t in ptrs}
    items = value.values() if isinstance(value, dict) else (value if isinstance(value, (tuple, list)) else (value,))
    for v in items:
        if isinstance(v, Tensor) and v.untyped_storage().data_ptr() in ptrs:
            return True
        if not isinstance(v, Tensor) and not isinstance(v, (int, float, bool, type(None))):
            return True  # nested structure: be conservative
    return False


class _MetricPendingSync:
    """Handle returned by ``Metric.sync(async_op=True)``; ``wait()`` installs the synchronised states."""

    def __init__(self, metric: "Metric", pending: Optional[PendingSync]) -> None:
        self._metric = metric
        self._pending = pending
        self._done = pending is None

    def wait(self) -> "Metric":
        if not self._done:
            self._metric._finish_async_sync(self._pending)
            self._done = True
        return self._metric
