"""Growable device arena behind list (``cat``) metric states.

The reference keeps a ``cat`` state as a Python list of tensors and concatenates it at every consumer
(``dim_zero_cat`` in compute, ``gather_all_tensors`` in sync: ``/root/reference/src/torchmetrics/utilities/data.py:28-36``,
``/root/reference/src/torchmetrics/metric.py:423-453``).  A metric whose value is read while it keeps accumulating
(``compute()`` every step, ``dist_sync_on_step``, ``MetricTracker``) therefore re-concatenates everything it has seen
at every read: O(steps^2) bytes over an epoch.

``StateArena`` is still a ``list`` (checkpoints, ``isinstance`` checks, user code that inspects ``metric.preds`` are
unchanged), but its first concatenation *compacts* the pieces into one buffer and turns the list items into views of
it.  Later appends are copied into the buffer's free tail while it has room, so the next concatenation is a view of
the filled prefix (no copy, no per-piece launches); when the tail is full the appended tensors are kept as they are
(zero-copy, like a plain list) and the next concatenation compacts again into a buffer of at least twice the
previous capacity.  Over any sequence of appends and reads every sample is copied O(1) times amortised.

* The first compaction allocates exactly the filled size (a single read never costs more HBM than ``torch.cat``).
* Pieces that differ in dtype / device / trailing shape, or that require grad, keep the plain-list behaviour.
* Any list mutation other than ``append`` / ``extend`` drops the buffer (the next read compacts again).
* ``cat()`` returns a view of the state; internal consumers treat it as read-only, as they treat a tensor state.
  ``Metric.compute`` copies any result that aliases an arena buffer before handing it to the user (the reference's
  ``dim_zero_cat`` always returns a fresh ``torch.cat``).
"""
from copy import deepcopy
from typing import Any, Iterable, List, Optional, Tuple

import torch
from torch import Tensor


class StateArena(list):
    """A list of tensors with a lazily compacted, growable backing buffer (see module docstring)."""

    __slots__ = ("_buf", "_rows", "_covered", "clean")

    def __init__(self, items: Iterable[Any] = ()) -> None:
        super().__init__(items)
        self._buf: Optional[Tensor] = None  # [capacity, *tail]
        self._rows = 0  # rows of _buf in use
        self._covered = 0  # list items [0, _covered) are views of _buf, in order
        # leading items a consumer has already filtered (CatMetric's deferred NaN drop); owned by this object, so it
        # cannot leak to a later arena the way an id()-keyed mark could
        self.clean = 0

    # ---------------------------------------------------------------------------------------------- helpers
    @staticmethod
    def _rows_of(t: Tensor) -> Tuple[int, Tuple[int, ...]]:
        return (1, ()) if t.ndim == 0 else (t.shape[0], tuple(t.shape[1:]))

    def _fits(self, t: Any) -> bool:
        buf = self._buf
        if buf is None or not isinstance(t, Tensor) or t.requires_grad:
            return False
        if t.dtype != buf.dtype or t.device != buf.device:
            return False
        rows, tail = self._rows_of(t)
        return tail == tuple(buf.shape[1:]) and self._rows + rows <= buf.shape[0]

    def _drop(self) -> None:
        self._buf, self._rows, self._covered = None, 0, 0

    def _compactable(self) -> bool:
        first = self[0]
        if not isinstance(first, Tensor):
            return False
        tail = self._rows_of(first)[1]
        for t in self:
            if not isinstance(t, Tensor) or t.requires_grad or t.dtype != first.dtype or t.device != first.device:
                return False
            if self._rows_of(t)[1] != tail:
                return False
        return True

    # ------------------------------------------------------------------------------------------ list protocol
    def append(self, t: Any) -> None:  # type: ignore[override]
        if self._covered == len(self) and self._fits(t):
            rows, _ = self._rows_of(t)
            dst = self._buf[self._rows : self._rows + rows]  # type: ignore[index]
            dst.copy_(t.reshape(dst.shape))
            super().append(dst.reshape(t.shape))
            self._rows += rows
            self._covered += 1
        else:
            super().append(t)

    def extend(self, items: Iterable[Any]) -> None:  # type: ignore[override]
        for t in items:
            self.append(t)

    def __iadd__(self, items: Iterable[Any]) -> "StateArena":  # type: ignore[override]
        self.extend(items)
        return self

    def _mutating(name: str):  # noqa: N805  (method factory)
        base = getattr(list, name)

        def method(self: "StateArena", *args: Any, **kwargs: Any) -> Any:
            self._drop()
            self.clean = 0
            return base(self, *args, **kwargs)

        method.__name__ = name
        return method

    __setitem__ = _mutating("__setitem__")
    __delitem__ = _mutating("__delitem__")
    insert = _mutating("insert")
    pop = _mutating("pop")
    remove = _mutating("remove")
    clear = _mutating("clear")
    sort = _mutating("sort")
    reverse = _mutating("reverse")
    del _mutating

    @classmethod
    def adopt(cls, other: "StateArena") -> "StateArena":
        """A new arena with ``other``'s items that takes over its buffer (and free tail); ``other`` keeps its items
        (views of the untouched prefix) but no longer appends into that buffer, so a list that is still shared
        elsewhere is never extended behind its holders' backs."""
        out = cls(other)
        out.clean = other.clean
        if other._buf is not None and other._covered == len(other):
            out._buf, out._rows, out._covered = other._buf, other._rows, other._covered
        other._drop()
        return out

    def truncate(self, k: int) -> None:
        """Drop the items from ``k`` on, keeping the buffer (and its free tail) when it covers the first ``k``."""
        k = max(0, min(k, len(self)))
        self.clean = min(self.clean, k)
        if self._buf is not None and self._covered >= k:
            self._rows = sum(self._rows_of(t)[0] for t in self[:k])
            self._covered = k
        else:
            self._drop()
        list.__delitem__(self, slice(k, None))

    # ------------------------------------------------------------------------------------------------ reads
    def cat(self) -> Tensor:
        """The concatenation along dim 0 (0-d items promoted to 1-d), as a view of the compacted buffer."""
        if not self:
            raise ValueError("No samples to concatenate")
        if self._buf is not None and self._covered == len(self):
            return self._buf[: self._rows]
        if not self._compactable():
            return torch.cat([t.unsqueeze(0) if t.ndim == 0 else t for t in self], dim=0)
        first = self[0]
        tail = self._rows_of(first)[1]
        total = sum(self._rows_of(t)[0] for t in self)
        cap = total if self._buf is None else max(total, 2 * self._buf.shape[0])
        buf = torch.empty((cap, *tail), dtype=first.dtype, device=first.device)
        pieces = [t.reshape(self._rows_of(t)[0], *tail) for t in self]
        torch.cat(pieces, dim=0, out=buf[:total])
        off = 0
        for i, t in enumerate(self):
            rows = self._rows_of(t)[0]
            list.__setitem__(self, i, buf[off : off + rows].reshape(t.shape))
            off += rows
        self._buf, self._rows, self._covered = buf, total, len(self)
        return buf[:total]

    def owns(self, t: Tensor) -> bool:
        """True if ``t`` is a view of this arena's buffer."""
        return self._buf is not None and t.untyped_storage().data_ptr() == self._buf.untyped_storage().data_ptr()

    @property
    def capacity(self) -> int:
        """Rows of the backing buffer (0 before the first compaction)."""
        return 0 if self._buf is None else int(self._buf.shape[0])

    # ------------------------------------------------------------------------------- copies and serialisation
    def compact_items(self) -> List[Any]:
        """Independent copies of the items (checkpoints hold one storage per item, as the reference's lists)."""
        return [t.detach().clone() if isinstance(t, Tensor) else deepcopy(t) for t in self]

    def __reduce_ex__(self, protocol: int) -> Any:
        return (StateArena, (self.compact_items(),))

    def __deepcopy__(self, memo: dict) -> "StateArena":
        out = StateArena()
        if self._buf is not None and self._covered == len(self) and all(not t.requires_grad for t in self):
            buf = self._buf.clone()
            off = 0
            for t in self:
                rows = self._rows_of(t)[0]
                list.append(out, buf[off : off + rows].reshape(t.shape))
                off += rows
            out._buf, out._rows, out._covered = buf, self._rows, len(self)
        else:
            list.extend(out, (deepcopy(t, memo) for t in self))
        out.clean = self.clean
        memo[id(self)] = out
        return out
