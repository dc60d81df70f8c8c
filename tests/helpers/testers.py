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


# ---------------------------------------------------------------------------------------------------------------
# further MetricTester checks (reference ``tests/unittests/helpers/testers.py:285-317, 454-520``)
# ---------------------------------------------------------------------------------------------------------------
def run_precision_test(
    preds: Tensor, target: Tensor, metric_class: Callable, metric_functional: Optional[Callable] = None,
    metric_args: Optional[Dict[str, Any]] = None, dtype: torch.dtype = torch.half, device: str = "cpu", atol: float = 5e-2,
) -> None:
    """Reduced-precision inputs: module (``update`` over the batches + ``compute``) and functional run, give finite
    results and agree with the fp32 run within ``atol``; the module's floating states may be ``set_dtype``-cast."""
    metric_args = metric_args or {}

    def cast(x: Tensor) -> Tensor:
        return x.to(dtype) if x.is_floating_point() else x

    ref_m = metric_class(**metric_args).to(device)
    low_m = metric_class(**metric_args).to(device)
    for i in range(len(preds)):
        ref_m.update(preds[i].to(device), target[i].to(device))
        low_m.update(cast(preds[i]).to(device), cast(target[i]).to(device))
    ref, low = _to_cpu(ref_m.compute()), _to_cpu(low_m.compute())
    assert_allclose(low, ref, atol)
    if metric_functional is not None:
        out = metric_functional(cast(preds[0]).to(device), cast(target[0]).to(device), **metric_args)
        ref_f = metric_functional(preds[0].to(device), target[0].to(device), **metric_args)
        assert_allclose(out, ref_f, atol)
    # set_dtype casts every floating state (and default, so reset keeps it); updates then follow the reference's
    # own promotion rules (e.g. Pearson's first batch mean takes the input dtype, as in the reference)
    cast_m = metric_class(**metric_args).to(device).set_dtype(torch.float64)
    for _ in range(2):
        for name, v in cast_m.metric_state.items():
            if isinstance(v, Tensor) and v.is_floating_point():
                assert v.dtype == torch.float64, (name, v.dtype)
        cast_m.update(preds[0].to(device), target[0].to(device))
        cast_m.reset()


def run_differentiability_test(
    preds: Tensor, target: Tensor, metric_class: Callable, metric_functional: Optional[Callable] = None,
    metric_args: Optional[Dict[str, Any]] = None,
) -> None:
    """``is_differentiable`` metrics propagate gradients to ``preds`` through ``forward`` and the functional; the
    others return results that do not require grad (reference ``run_differentiability_test``)."""
    metric_args = metric_args or {}
    metric = metric_class(**metric_args)
    p = preds[0].clone().to(torch.float64 if preds.is_floating_point() else preds.dtype)
    if not p.is_floating_point():
        return
    p.requires_grad_(True)
    out = metric(p, target[0])
    outs = [o for o in (out.values() if isinstance(out, dict) else (out if isinstance(out, (list, tuple)) else [out]))
            if isinstance(o, Tensor)]
    if metric.is_differentiable:
        assert any(o.requires_grad for o in outs), "is_differentiable metric returned no grad-carrying output"
        total = sum(o.double().sum() for o in outs if o.requires_grad)
        total.backward()
        assert p.grad is not None and torch.isfinite(p.grad).all()
        if metric_functional is not None:
            q = p.detach().clone().requires_grad_(True)
            metric_functional(q, target[0], **metric_args).double().sum().backward()
            assert q.grad is not None
    else:
        assert not any(o.requires_grad for o in outs), "non-differentiable metric returned a grad-carrying output"


def run_scriptable_test(metric_class: Callable, preds: Tensor, target: Tensor, metric_args: Optional[Dict[str, Any]] = None) -> None:
    """``torch.jit.script`` succeeds on a fresh and on an updated module (the reference's ``check_scriptable``), and
    scripting leaves the eager module's value unchanged."""
    metric_args = metric_args or {}
    torch.jit.script(metric_class(**metric_args))
    eager = metric_class(**metric_args)
    eager.update(preds[0], target[0])
    before = _to_cpu(eager.compute())
    torch.jit.script(eager)
    assert_allclose(eager.compute(), before, 0.0)
