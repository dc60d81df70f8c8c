"""Native op layer: hand-written gfx950 HIP kernels exposed as ``torch.ops.tmx.*``.

Policy (MI355X-first, no silent fallbacks on the GPU):

* ``load()`` loads ``_tmx_native.so`` (built in-tree by :mod:`.build`).  On a machine with a ROCm GPU the
  library **must** load: every GPU code path calls :func:`require`, which raises if it is missing, so a GPU run
  can never quietly degrade to eager PyTorch.
* CPU tensors (gloo / plumbing configs, unit tests in the CPU container) use the pure-PyTorch reference
  implementations that live next to each wrapper; these are also the numerics oracles for the kernel tests.
* Set ``TMX_DISABLE_NATIVE=1`` to force the eager path for A/B comparisons (documented, never implicit).
"""
import os
import threading
from pathlib import Path
from typing import Optional

import torch

# ``TMX_NATIVE_LIB`` points at an alternative build of the same ops (e.g. the ASan/UBSan host-only library of
# ``tools/sanitize_host.py``); default: the in-tree gfx950 library
_LIB = Path(os.environ.get("TMX_NATIVE_LIB") or Path(__file__).resolve().parent / "_tmx_native.so")
_lock = threading.Lock()
_loaded: Optional[bool] = None
_error: Optional[str] = None


# read once at import (A/B switch for whole processes); use_native runs on every update's hot path
_DISABLED = os.environ.get("TMX_DISABLE_NATIVE", "0") == "1"


def load() -> bool:
    """Load the native library once; returns True on success."""
    global _loaded, _error
    if _loaded is not None:
        return _loaded
    with _lock:
        if _loaded is not None:
            return _loaded
        if os.environ.get("TMX_DISABLE_NATIVE", "0") == "1":
            _loaded, _error = False, "disabled by TMX_DISABLE_NATIVE=1"
            return False
        if not _LIB.exists():
            _loaded, _error = False, f"{_LIB} not built (run `python -m torchmetrics_forked_amd.ops.build`)"
            return False
        try:
            torch.ops.load_library(str(_LIB))
            _loaded = True
        except Exception as err:  # pragma: no cover - surfaced through require()
            _loaded, _error = False, f"failed to load {_LIB}: {err}"
    return bool(_loaded)


def available() -> bool:
    return load()


_py_mod: Optional[object] = None


def py_module() -> Optional[object]:
    """The library's CPython entry point (``csrc/py_columns.cpp``: host helpers that read Python containers in C,
    where a ``torch.ops`` call would box every tensor of a list); ``None`` when the library is not loaded."""
    global _py_mod
    if _py_mod is None and load():
        import importlib.util

        spec = importlib.util.spec_from_file_location("_tmx_native", str(_LIB))
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        _py_mod = mod
    return _py_mod


def require(tensor: Optional[torch.Tensor] = None) -> None:
    """Raise unless the native library is loaded (called on every GPU code path)."""
    if not load():
        where = f" for a tensor on {tensor.device}" if tensor is not None else ""
        raise RuntimeError(f"torchmetrics_forked_amd native HIP library required{where}: {_error}")


def _device_error(a: torch.device, b: torch.device) -> RuntimeError:
    return RuntimeError(f"Expected all tensors to be on the same device, but found at least two devices, {a} and {b}!")


def use_native(t: torch.Tensor, *others: Optional[torch.Tensor]) -> bool:
    """True when ``t`` lives on the GPU; then the native library is mandatory (raises if missing).

    ``others``: every further tensor the native call would read or write.  They must sit on ``t``'s device (0-dim
    host scalars excepted): a HIP kernel handed a host pointer faults the GPU instead of raising, so the device error
    torch itself would give is raised here, before any launch."""
    if t.is_cuda:
        dev = t.device
        for o in others:
            if o is not None and o.device != dev and not (o.device.type == "cpu" and o.dim() == 0):
                raise _device_error(dev, o.device)
        if _DISABLED:
            return False
        if not _loaded:
            require(t)
        return True
    for o in others:
        if isinstance(o, torch.Tensor) and o.is_cuda:
            raise _device_error(o.device, t.device)
    return False


def lib_path() -> Path:
    return _LIB
