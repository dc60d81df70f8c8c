"""Eager vs deferred tensor validation.

The reference validates every ``update`` with host-synchronising checks (``torch.unique`` + Python ``if``,
SURVEY §0 fact 6).  On MI355X that stalls the HIP stream once or twice per step.  Here a validator receives a
``sink``:

* ``sink is None`` (functional API, CPU tensors, or ``TMX_VALIDATION=eager``): raise immediately, exactly like the
  reference (same exception types and messages).
* ``sink`` is a :class:`DeferredChecks` (module metrics on GPU tensors): each check contributes a device-side
  boolean flag; flags are OR-ed on device and inspected once, at ``compute`` time (which synchronises anyway),
  raising the same exception type and message.
"""
import os
import warnings
from typing import Callable, Dict, List, Optional, Tuple, Type

import torch
from torch import Tensor


def validation_mode() -> str:
    return os.environ.get("TMX_VALIDATION", "auto")


class DeferredChecks:
    """Accumulates device-side failure flags keyed by (exception type, message).

    Two ways to contribute: ``add(bad, ...)`` ORs a boolean tensor in (one small reduction kernel), or
    ``flag(...)`` hands out a persistent ``int32[1]`` device word that native kernels OR into directly while
    they stream the data anyway (zero extra kernels per update).
    """

    def __init__(self) -> None:
        self._flags: Dict[Tuple[Type[Exception], str], Tensor] = {}

    def add(self, bad: Tensor, exc: Type[Exception], message: str) -> None:
        key = (exc, message)
        bad = bad.reshape(-1).any().reshape(1).to(torch.int32)
        prev = self._flags.get(key)
        if prev is None:
            self._flags[key] = bad
        else:
            prev.bitwise_or_(bad)

    def flag(self, exc: Type[Exception], message: str, device: torch.device) -> Tensor:
        key = (exc, message)
        f = self._flags.get(key)
        if f is None or f.device != device:
            f = torch.zeros(1, dtype=torch.int32, device=device)
            self._flags[key] = f
        return f

    def attach(self, exc: Type[Exception], message: str, flag: Tensor) -> None:
        """Share another sink's device flag (one kernel writes, several metrics raise)."""
        self._flags[(exc, message)] = flag

    def check(self) -> None:
        if not self._flags:
            return
        keys = list(self._flags.keys())
        flags = torch.cat([self._flags[k].reshape(1).to(torch.int32).cpu() for k in keys])  # one host sync
        for k in keys:
            self._flags[k].zero_()
        errors = []
        for k, f in zip(keys, flags.tolist()):
            if f:
                if issubclass(k[0], Warning):  # deferred warnings (e.g. aggregation nan_strategy="warn")
                    warnings.warn(k[1], k[0], stacklevel=3)
                else:
                    errors.append(k)
        if errors:
            raise errors[0][0](errors[0][1])

    def clear(self) -> None:
        for f in self._flags.values():
            f.zero_()


def make_sink(t: Tensor) -> Optional[DeferredChecks]:
    """Sink for a tensor: deferred on GPU (unless TMX_VALIDATION=eager), eager otherwise."""
    mode = validation_mode()
    if mode == "eager" or (mode == "auto" and not t.is_cuda):
        return None
    return DeferredChecks()


def fail_if(
    bad: Tensor,
    exc: Type[Exception],
    message: Callable[[], str],
    sink: Optional[DeferredChecks],
    static_message: Optional[str] = None,
) -> None:
    """Raise ``exc(message())`` if ``bad`` (eager) or record it in ``sink`` (deferred).

    ``message`` may read tensor values (only evaluated when raising eagerly); deferred mode uses
    ``static_message`` (no host access) or a generic description.
    """
    if sink is None:
        if bool(bad.any()):
            raise exc(message())
    else:
        sink.add(bad, exc, static_message or "Invalid input values detected (deferred validation at compute).")
