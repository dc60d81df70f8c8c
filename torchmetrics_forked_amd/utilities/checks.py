"""Input checks (parity: reference ``utilities/checks.py``).

The framework's classification validators live next to the formatting code (``functional/classification``);
this module keeps the shared, domain-agnostic checks plus ``check_forward_full_state_property``.
"""
import os
import time
from functools import partial
from typing import Any, Callable, Dict, Mapping, Optional, Sequence, Tuple

import torch
from torch import Tensor

_DOCTEST_DOWNLOAD_TIMEOUT = int(os.environ.get("DOCTEST_DOWNLOAD_TIMEOUT", 120))
_SKIP_SLOW_DOCTEST = bool(os.environ.get("SKIP_SLOW_DOCTEST", 0))


def _check_for_empty_tensors(preds: Tensor, target: Tensor) -> bool:
    return preds.numel() == target.numel() == 0


def _check_same_shape(preds: Tensor, target: Tensor) -> None:
    if preds.shape != target.shape:
        raise RuntimeError(
            f"Predictions and targets are expected to have the same shape, but got {preds.shape} and {target.shape}."
        )


def _check_retrieval_target_and_prediction_types(
    preds: Tensor, target: Tensor, allow_non_binary_target: bool = False, sink: Optional[Any] = None
) -> Tuple[Tensor, Tensor]:
    """``sink`` (a ``DeferredChecks``): the binary-target check becomes a device flag raised at ``compute`` instead
    of two host synchronisations per update; bool targets are binary by construction and skip it."""
    if target.dtype not in (torch.bool, torch.long, torch.int) and not torch.is_floating_point(target):
        raise ValueError("`target` must be a tensor of booleans, integers or floats")
    if not preds.is_floating_point():
        raise ValueError("`preds` must be a tensor of floats")
    if not allow_non_binary_target and target.dtype != torch.bool:
        if sink is None:
            if target.max() > 1 or target.min() < 0:
                raise ValueError("`target` must contain `binary` values")
        else:
            sink.add((target > 1) | (target < 0), ValueError, "`target` must contain `binary` values")
    target = target.float() if target.is_floating_point() else target.long()
    return preds.float().flatten(), target.flatten()


def _check_retrieval_functional_inputs(
    preds: Tensor, target: Tensor, allow_non_binary_target: bool = False
) -> Tuple[Tensor, Tensor]:
    if preds.shape != target.shape:
        raise ValueError("`preds` and `target` must be of the same shape")
    if not preds.numel() or not preds.size():
        raise ValueError("`preds` and `target` must be non-empty and non-scalar tensors")
    return _check_retrieval_target_and_prediction_types(preds, target, allow_non_binary_target)


def _check_retrieval_inputs(
    indexes: Tensor,
    preds: Tensor,
    target: Tensor,
    allow_non_binary_target: bool = False,
    ignore_index: Optional[int] = None,
    sink: Optional[Any] = None,
) -> Tuple[Tensor, Tensor, Tensor]:
    if indexes.shape != preds.shape or preds.shape != target.shape:
        raise ValueError("`indexes`, `preds` and `target` must be of the same shape")
    if indexes.dtype is not torch.long:
        raise ValueError("`indexes` must be a tensor of long integers")
    if ignore_index is not None:
        keep = target != ignore_index
        indexes, preds, target = indexes[keep], preds[keep], target[keep]
    if not indexes.numel() or not indexes.size():
        raise ValueError("`indexes`, `preds` and `target` must be non-empty and non-scalar tensors")
    preds, target = _check_retrieval_target_and_prediction_types(preds, target, allow_non_binary_target, sink)
    return indexes.long().flatten(), preds, target


def _allclose_recursive(res1: Any, res2: Any, atol: float = 1e-6) -> bool:
    if isinstance(res1, Tensor):
        return torch.allclose(res1, res2, atol=atol)
    if isinstance(res1, str):
        return res1 == res2
    if isinstance(res1, Sequence):
        return all(_allclose_recursive(a, b) for a, b in zip(res1, res2))
    if isinstance(res1, Mapping):
        return all(_allclose_recursive(res1[k], res2[k]) for k in res1)
    return res1 == res2


def check_forward_full_state_property(
    metric_class: Any,
    init_args: Optional[Dict[str, Any]] = None,
    input_args: Optional[Dict[str, Any]] = None,
    num_update_to_compare: Sequence[int] = (10, 100, 1000),
    reps: int = 5,
) -> None:
    """Check whether ``full_state_update=False`` is safe for ``metric_class`` and report the speed-up.

    Two subclasses are built (full / reduce state forward); their per-step outputs must match, then both
    are timed for several update counts (parity: reference ``utilities/checks.py:636-738``).
    """
    init_args = init_args or {}
    input_args = input_args or {}

    class FullState(metric_class):
        full_state_update = True

    class PartState(metric_class):
        full_state_update = False

    fullstate = FullState(**init_args)
    partstate = PartState(**init_args)
    equal = True
    try:
        for _ in range(num_update_to_compare[0]):
            equal = equal & _allclose_recursive(fullstate(**input_args), partstate(**input_args))
    except RuntimeError:
        equal = False
    res1, res2 = fullstate.compute(), partstate.compute()
    equal = equal & _allclose_recursive(res1, res2)
    if not equal:
        print("Full state for this metric is necessary. Full state update and partial state update gave different results.")
        return

    mean = torch.zeros(2, len(num_update_to_compare))
    std = torch.zeros(2, len(num_update_to_compare))
    for i, n in enumerate(num_update_to_compare):
        for j, m_cls in enumerate((FullState, PartState)):
            times = []
            for _ in range(reps):
                metric = m_cls(**init_args)
                start = time.perf_counter()
                for _ in range(n):
                    metric(**input_args)
                times.append(time.perf_counter() - start)
            mean[j, i] = torch.tensor(times).mean()
            std[j, i] = torch.tensor(times).std()
    for i, n in enumerate(num_update_to_compare):
        print(f"Full state for {n} steps took: {mean[0, i]:0.3f}+-{std[0, i]:0.3f}")
        print(f"Partial state for {n} steps took: {mean[1, i]:0.3f}+-{std[1, i]:0.3f}")
    faster = (mean[1, -1] < mean[0, -1]).item()
    print(f"Recommended setting `full_state_update={not faster}`")


def is_overridden(method_name: str, instance: object, parent: object) -> bool:
    instance_attr = getattr(instance, method_name, None)
    if instance_attr is None:
        return False
    if hasattr(instance_attr, "__wrapped__"):
        instance_attr = instance_attr.__wrapped__
    if isinstance(instance_attr, partial):
        instance_attr = instance_attr.func
    parent_attr = getattr(parent, method_name, None)
    if parent_attr is None:
        raise ValueError("The parent should define the method")
    return getattr(instance_attr, "__code__", None) is not getattr(parent_attr, "__code__", None)


def _try_proceed_with_timeout(fn: Callable, timeout: int = _DOCTEST_DOWNLOAD_TIMEOUT) -> bool:
    """Run ``fn`` in a worker thread; False if it did not finish in ``timeout`` seconds (offline-safe)."""
    import threading

    done = threading.Event()

    def _run() -> None:
        try:
            fn()
        finally:
            done.set()

    threading.Thread(target=_run, daemon=True).start()
    return done.wait(timeout)
