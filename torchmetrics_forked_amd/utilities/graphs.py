"""HIP-graph replay of metric updates (the MI355X answer to launch-bound small batches).

A metric update on a small batch (BASELINE config 1: ``MulticlassAccuracy``, C=5, batch 10) costs a handful of
kernel launches plus the Python around them, tens of microseconds of host time for microseconds of GPU work.  The
reference has no answer to this except "use bigger batches"; here ``GraphedUpdate`` captures one
``Metric.update`` / ``MetricCollection.update`` into a HIP graph (``torch.cuda.CUDAGraph`` on ROCm) and replays it
for every later batch of the same shapes: one graph launch, no Python in the kernels' path.

Requirements (checked, with a clear error instead of wrong numbers):
  * every argument tensor is on the GPU, and later batches have the same shapes / dtypes (they are copied into
    the captured input buffers);
  * the update has no host synchronisation (the common GPU updates of this package have none: input checks are
    deferred device flags, see ``utilities/validation.py``);
  * every state is a tensor updated IN PLACE (native kernels accumulate into the state; ``self.x += y`` works,
    ``self.x = self.x + y`` would rebind the state to graph-private memory and is rejected); list (``cat``)
    states cannot be captured.

Warm-up updates run on a side stream before capture (as for any graph capture) and are rolled back: states and
deferred-check flags are restored, so the graphed metric holds exactly the replayed batches.

The graph writes into the storage the states had at capture time.  ``reset()``, ``forward()``, ``.to()`` and
``load_state_dict`` rebind states to new tensors, so every replay first compares the members' current state and flag
storages with the captured ones and re-captures (same warm-up and roll-back) when any of them moved: the usual
``compute(); reset()`` epoch loop keeps accumulating into the live states instead of into orphaned buffers.
"""
from typing import Any, Dict, List, Tuple, Union

import torch
from torch import Tensor

from torchmetrics_forked_amd.collections import MetricCollection
from torchmetrics_forked_amd.metric import Metric


def _members(obj: Union[Metric, MetricCollection]) -> List[Metric]:
    if isinstance(obj, MetricCollection):
        return list(obj.values(copy_state=False))
    return [obj]


def _flatten_inputs(args: Tuple[Any, ...], kwargs: Dict[str, Any]) -> List[Tensor]:
    flat = [a for a in args if isinstance(a, Tensor)] + [v for v in kwargs.values() if isinstance(v, Tensor)]
    for t in flat:
        if not t.is_cuda:
            raise ValueError("GraphedUpdate needs GPU input tensors")
    return flat


class GraphedUpdate:
    """Capture ``metric.update(*example_args, **example_kwargs)`` once; ``self(*args, **kwargs)`` replays it.

    Args:
        metric: a ``Metric`` or ``MetricCollection`` whose states live on the GPU.
        example_args / example_kwargs: a batch with the shapes and dtypes of every later batch (its values are not
            accumulated). Non-tensor arguments are frozen at capture time.
        warmup: side-stream warm-up updates before capture (rolled back).

    Example (needs a GPU)::

        coll = tm.MetricCollection({"acc": tm.MulticlassAccuracy(num_classes=10),
                                    "ece": tm.MulticlassCalibrationError(num_classes=10),
                                    "cm": tm.MulticlassConfusionMatrix(num_classes=10)}, compute_groups=False).cuda()
        step = GraphedUpdate(coll, logits, labels)   # example batch: shapes / dtypes only
        for logits, labels in loader:                # same shapes every step
            step(logits, labels)                     # one graph replay instead of the eager update
        coll.compute()
    """

    def __init__(self, metric: Union[Metric, MetricCollection], *example_args: Any, warmup: int = 2, **example_kwargs: Any) -> None:
        if not torch.cuda.is_available():
            raise RuntimeError("GraphedUpdate needs a GPU")
        self.metric = metric
        self._warmup = warmup
        inputs = _flatten_inputs(example_args, example_kwargs)
        self._static_args = tuple(a.clone() if isinstance(a, Tensor) else a for a in example_args)
        self._static_kwargs = {k: (v.clone() if isinstance(v, Tensor) else v) for k, v in example_kwargs.items()}
        self._static_inputs = _flatten_inputs(self._static_args, self._static_kwargs)
        self._shapes = [(t.shape, t.dtype) for t in inputs]
        self._device = inputs[0].device if inputs else torch.device("cuda", torch.cuda.current_device())
        self.captures = 0
        self._capture()

    def _capture(self) -> None:
        """Warm up on a side stream, roll back, capture one update; records the storages the graph writes."""
        metric, warmup, device = self.metric, self._warmup, self._device
        self._members = _members(metric)
        counts = [m._update_count for m in self._members]
        lists = self._list_lengths()
        states = self._tensor_states()
        saved = {key: t.clone() for key, t in states.items()}
        saved_flags = self._flag_values()

        side = torch.cuda.Stream(device=device)
        side.wait_stream(torch.cuda.current_stream(device))
        with torch.cuda.stream(side):
            for _ in range(max(warmup, 1)):  # first updates may create lazy buffers / flags / compute groups
                metric.update(*self._static_args, **self._static_kwargs)
        torch.cuda.current_stream(device).wait_stream(side)
        for m in self._members:  # work the warm-up left on other streams (curve update lanes) lands before the roll-back
            m._join_side_work()

        # the state tensors the warm-up left are the ones the graph accumulates into (a fresh collection may merge
        # its compute groups' states during its first update, so states can be rebound here, not during capture)
        after = self._tensor_states()
        self._restore(after, saved, saved_flags)
        if self._list_lengths() != lists:
            self._reset_counts(counts)
            raise ValueError(
                f"GraphedUpdate: {type(metric).__name__}.update appends to a list (`cat`) state; only tensor states"
                " updated in place can be captured"
            )

        graph = torch.cuda.CUDAGraph()
        try:
            with torch.cuda.graph(graph):
                metric.update(*self._static_args, **self._static_kwargs)
        except RuntimeError as err:
            self._restore(after, saved, saved_flags)
            self._reset_counts(counts)
            raise RuntimeError(
                f"GraphedUpdate: {type(metric).__name__}.update could not be captured into a HIP graph (host"
                f" synchronisation or an unsupported op inside update): {err}"
            ) from err
        self._check_in_place(after, self._tensor_states(), "capture")
        for m in self._members:  # host-side accounting that replays cannot advance is switched to its safe mode
            hook = getattr(m, "_after_graph_capture", None)
            if hook is not None:
                hook()
        self._graph = graph
        self._reset_counts(counts)
        self._ptrs = self._storage_ptrs()
        self.captures += 1
        torch.cuda.synchronize(device)

    # -------------------------------------------------------------------------------------------- helpers
    def _tensor_states(self) -> Dict[Tuple[int, str], Tensor]:
        out: Dict[Tuple[int, str], Tensor] = {}
        for i, m in enumerate(self._members):
            for name in m._defaults:
                val = getattr(m, name)
                if isinstance(val, list):  # list states must stay untouched (e.g. the sample lists of a histogram curve)
                    continue
                if not val.is_cuda:
                    raise ValueError(f"GraphedUpdate: state `{name}` of {type(m).__name__} is not on the GPU")
                out[(i, name)] = val
        return out

    def _storage_ptrs(self) -> List[int]:
        """Data pointers of every tensor state and deferred-check flag the graph writes (plus the member identities)."""
        members = _members(self.metric)
        ptrs: List[int] = [id(m) for m in members]
        for m in members:
            for name in m._defaults:
                val = getattr(m, name)
                if isinstance(val, Tensor):
                    ptrs.append(val.data_ptr())
            d = m._deferred
            if d is not None:
                ptrs.extend(f.data_ptr() for f in d._flags.values())
        return ptrs

    def _list_lengths(self) -> List[int]:
        return [len(getattr(m, n)) for m in self._members for n in m._defaults if isinstance(getattr(m, n), list)]

    def _check_in_place(self, before: Dict[Tuple[int, str], Tensor], after: Dict[Tuple[int, str], Tensor], when: str) -> None:
        for key, t in before.items():
            if after[key].data_ptr() != t.data_ptr():
                m = self._members[key[0]]
                raise ValueError(
                    f"GraphedUpdate: {type(m).__name__}.update rebinds state `{key[1]}` during {when} instead of"
                    " updating it in place; a replayed graph would not accumulate it"
                )

    def _flag_values(self) -> Dict[Tuple[int, Any], Tensor]:
        vals = {}
        for i, m in enumerate(self._members):
            d = m._deferred
            if d is not None:
                for key, f in d._flags.items():
                    vals[(i, key)] = f.clone()
        return vals

    def _restore(self, states: Dict[Tuple[int, str], Tensor], saved: Dict[Tuple[int, str], Tensor],
                 saved_flags: Dict[Tuple[int, Any], Tensor]) -> None:
        with torch.no_grad():
            for key, t in states.items():
                old = saved[key]
                if old.shape == t.shape:
                    t.copy_(old)
                else:  # created lazily by the warm-up (e.g. a histogram state that starts empty): no data yet
                    t.zero_()
            for i, m in enumerate(self._members):
                d = m._deferred
                if d is None:
                    continue
                for key, f in d._flags.items():
                    old = saved_flags.get((i, key))
                    f.copy_(old) if old is not None else f.zero_()

    def _reset_counts(self, counts: List[int]) -> None:
        for m, c in zip(self._members, counts):
            m._update_count = c
            m._computed = None

    # ----------------------------------------------------------------------------------------------- replay
    def __call__(self, *args: Any, **kwargs: Any) -> None:
        """Accumulate one batch (same shapes / dtypes as the example) by replaying the captured update."""
        inputs = _flatten_inputs(args, kwargs)
        if [(t.shape, t.dtype) for t in inputs] != self._shapes:
            raise ValueError(
                f"GraphedUpdate: batch shapes {[(tuple(t.shape), t.dtype) for t in inputs]} differ from the captured"
                f" {[(tuple(s), d) for s, d in self._shapes]}"
            )
        if self._storage_ptrs() != self._ptrs:
            # reset() / forward() / .to() / load_state_dict rebound a state or flag: the captured graph would add into
            # the old storage, so capture again against the live one
            self._graph = None
            self._capture()
        for dst, src in zip(self._static_inputs, inputs):
            dst.copy_(src, non_blocking=True)
        self._graph.replay()
        for m in self._members:
            m._update_count += 1
            m._computed = None
