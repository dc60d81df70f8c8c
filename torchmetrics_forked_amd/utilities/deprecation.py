"""Deprecated root-level import shims (behaviour of the reference's ``*/_deprecated.py`` modules).

Importing a domain metric from the package root (``torchmetrics_forked_amd.BLEUScore``) or a domain function from
``torchmetrics_forked_amd.functional`` still works but emits a ``FutureWarning`` pointing at the domain package,
exactly like the reference (e.g. reference ``text/_deprecated.py``, ``functional/text/_deprecated.py``).  The shims
are generated from the real classes / functions, so signatures and behaviour are identical."""
import functools
from typing import Any, Callable, Type

from torchmetrics_forked_amd.utilities.prints import _deprecated_root_import_class, _deprecated_root_import_func


def deprecated_class(cls: Type, domain: str) -> Type:
    """Subclass of ``cls`` named ``_<Name>`` whose constructor warns about the root import."""

    def __init__(self: Any, *args: Any, **kwargs: Any) -> None:
        _deprecated_root_import_class(cls.__name__, domain)
        cls.__init__(self, *args, **kwargs)

    shim = type(f"_{cls.__name__}", (cls,), {"__init__": __init__, "__doc__": f"Wrapper for deprecated import of ``{cls.__name__}``."})
    shim.__module__ = cls.__module__
    return shim


def deprecated_func(fn: Callable, domain: str) -> Callable:
    """Wrapper of ``fn`` named ``_<name>`` that warns about the ``functional`` root import."""

    @functools.wraps(fn)
    def wrapper(*args: Any, **kwargs: Any) -> Any:
        _deprecated_root_import_func(fn.__name__, domain)
        return fn(*args, **kwargs)

    wrapper.__name__ = f"_{fn.__name__}"
    return wrapper
