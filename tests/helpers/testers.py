"""MetricTester-style harness (test strategy mirrors reference ``tests/unittests/helpers/testers.py``).

``run_class_metric_test`` checks, on 1 process or on the 2-process gloo pool:
  * constant class attributes cannot be set, ``clone``/pickle round-trips, hashing, empty default state_dict;
  * strided batch sharding ``range(rank, num_batches, world)``; per-batch ``forward`` values vs the oracle (on the
    rank-local batch, or on all ranks' batches when ``dist_sync_on_step``);
  * final ``compute()`` vs the oracle on *all* batches (exercises the coalesced sync engine).
"""
import pickle
from copy import deepcopy
from typing import Any, Callable, Dict, Optional, Sequence

import numpy as np
import torch
from torch import Tensor

from tests.helpers.ddp import NUM_PROCESSES, run_ddp

NUM_BATCHES = 4
BATCH_SIZE = 32
NUM_CLASSES = 5
EXTRA_DIM = 3
THRESHOLD = 0.5


def _to_cpu(x: Any) -> Any:
    if isinstance(x, Tensor):
        return x.detach().cpu()
    if isinstance(x, dict):
        return {k: _to_cpu(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return type(x)(_to_cpu(v) for v in x)
    return x


def assert_allclose(res: Any, ref: Any, atol: float = 1e-6, key: Optional[str] = None) -> None:
    res, ref = _to_cpu(res), _to_cpu(ref)
    if isinstance(res, dict):
        if key is None:
            for k in res:
                assert_allclose(res[k], ref[k], atol)
            return
        res = res[key]
    if isinstance(res, (list, tuple)):
        assert len(res) == len(ref), (len(res), len(ref))
        for a, b in zip(res, ref):
            assert_allclose(a, b, atol)
        return
    if isinstance(res, Tensor) or isinstance(ref, Tensor):
        a = torch.as_tensor(res, dtype=torch.float64)
        b = torch.as_tensor(np.asarray(ref) if not isinstance(ref, Tensor) else ref, dtype=torch.float64)
        assert a.shape == b.shape or a.numel() == b.numel(), (a.shape, b.shape)
        assert torch.allclose(a.reshape(b.shape), b, atol=atol, equal_nan=True), f"\n{a}\nvs\n{b}"
        return
    np.testing.assert_allclose(res, ref, atol=atol)


def _class_test(
    rank: int,
    world: int,
    preds: Any,
    target: Any,
    metric_class: Callable,
    reference_metric: Callable,
    metric_args: Dict[str, Any],
    dist_sync_on_step: bool,
    check_batch: bool,
    atol: float,
    device: str,
    fragment_kwargs: bool,
    check_state_dict: bool,
) -> None:
    metric = metric_class(**metric_args, dist_sync_on_step=dist_sync_on_step).to(device)
    for attr in ("higher_is_better", "is_differentiable", "full_state_update"):
        try:
            setattr(metric, attr, True)
            raise AssertionError(f"const attribute {attr} was settable")
        except RuntimeError:
            pass
    metric_clone = deepcopy(metric)
    metric = pickle.loads(pickle.dumps(metric_clone))
    hash(metric)
    if check_state_dict:
        assert metric.state_dict() == {} or all(not v for v in metric._persistent.values())

    num_batches = len(preds)
    for i in range(rank, num_batches, world):
        p, t = preds[i], target[i]
        p = p.to(device) if isinstance(p, Tensor) else p
        t = t.to(device) if isinstance(t, Tensor) else t
        batch_result = metric(p, t)
        if metric.dist_sync_on_step and check_batch and world > 1:
            idx = [j for j in range(i - rank, i - rank + world) if j < num_batches]
            if len(idx) == world:
                ref = reference_metric(_cat([preds[j] for j in idx]), _cat([target[j] for j in idx]))
                assert_allclose(batch_result, ref, atol)
        elif check_batch and not metric.dist_sync_on_step:
            assert_allclose(batch_result, reference_metric(preds[i], target[i]), atol)
    result = metric.compute()
    # gathered `cat` states are rank-major: order the oracle input the same way
    order = [i for r in range(world) for i in range(r, num_batches, world)]
    ref = reference_metric(_cat([preds[i] for i in order]), _cat([target[i] for i in order]))
    assert_allclose(result, ref, atol)


def _cat(xs: Sequence[Any]) -> Any:
    if isinstance(xs[0], Tensor):
        return torch.cat(xs, 0)
    out: list = []
    for x in xs:
        out.extend(x)
    return out


def run_class_metric_test(
    ddp: bool,
    preds: Any,
    target: Any,
    metric_class: Callable,
    reference_metric: Callable,
    metric_args: Optional[Dict[str, Any]] = None,
    dist_sync_on_step: bool = False,
    check_batch: bool = True,
    atol: float = 1e-6,
    device: str = "cpu",
    fragment_kwargs: bool = False,
    check_state_dict: bool = True,
) -> None:
    args = (preds, target, metric_class, reference_metric, metric_args or {}, dist_sync_on_step, check_batch, atol, device,
            fragment_kwargs, check_state_dict)
    if ddp:
        run_ddp(_class_test, *args)
    else:
        _class_test(0, 1, *args)


def run_functional_metric_test(
    preds: Any, target: Any, metric_functional: Callable, reference_metric: Callable,
    metric_args: Optional[Dict[str, Any]] = None, atol: float = 1e-6, device: str = "cpu",
) -> None:
    metric_args = metric_args or {}
    for i in range(len(preds)):
        p = preds[i].to(device) if isinstance(preds[i], Tensor) else preds[i]
        t = target[i].to(device) if isinstance(target[i], Tensor) else target[i]
        assert_allclose(metric_functional(p, t, **metric_args), reference_metric(preds[i], target[i]), atol)


class RefFn:
    """Picklable reference-oracle callable: ``torchmetrics.functional.<...>.<name>(p, t, **kwargs)`` from the
    read-only reference (imported lazily, also inside spawned DDP workers)."""

    def __init__(self, name: str, domain: str = "classification", **kwargs: Any) -> None:
        self.name, self.domain, self.kwargs = name, domain, kwargs

    def __call__(self, p: Any, t: Any) -> Any:
        import sys

        for path in ("/root/repo/tests/_oracle", "/root/reference/src"):
            if path not in sys.path:
                sys.path.append(path)
        import importlib

        mod = importlib.import_module(f"torchmetrics.functional.{self.domain}" if self.domain else "torchmetrics.functional")
        return getattr(mod, self.name)(p, t, **self.kwargs)
