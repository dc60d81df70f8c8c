"""Rank-zero logging helpers (behavioural parity with reference ``utilities/prints.py:22-73``).

Rank is resolved lazily from ``RANK``/``LOCAL_RANK`` so that ``torchrun`` children that import the package
before the process group exists still log only once per node.
"""
import logging
import os
import warnings
from functools import partial, wraps
from typing import Any, Callable

log = logging.getLogger("torchmetrics_forked_amd")


def _current_rank() -> int:
    for key in ("LOCAL_RANK", "RANK"):
        val = os.environ.get(key)
        if val is not None:
            try:
                return int(val)
            except ValueError:
                return 0
    return 0


def rank_zero_only(fn: Callable) -> Callable:
    """Decorate ``fn`` so it only executes on (local) rank zero."""

    @wraps(fn)
    def wrapped(*args: Any, **kwargs: Any) -> Any:
        if _current_rank() == 0:
            return fn(*args, **kwargs)
        return None

    return wrapped


def _warn(*args: Any, **kwargs: Any) -> None:
    kwargs.setdefault("stacklevel", 4)
    warnings.warn(*args, **kwargs)


def _info(*args: Any, **kwargs: Any) -> None:
    log.info(*args, **kwargs)


def _debug(*args: Any, **kwargs: Any) -> None:
    log.debug(*args, **kwargs)


rank_zero_debug = rank_zero_only(_debug)
rank_zero_info = rank_zero_only(_info)
rank_zero_warn = rank_zero_only(_warn)
_future_warning = partial(warnings.warn, category=FutureWarning)


def _deprecated_root_import_class(name: str, domain: str) -> None:
    _future_warning(
        f"Importing `{name}` from `torchmetrics_forked_amd` was deprecated and will be removed in 2.0."
        f" Import `{name}` from `torchmetrics_forked_amd.{domain}` instead."
    )


def _deprecated_root_import_func(name: str, domain: str) -> None:
    _future_warning(
        f"Importing `{name}` from `torchmetrics_forked_amd.functional` was deprecated and will be removed in 2.0."
        f" Import `{name}` from `torchmetrics_forked_amd.{domain}` instead."
    )
