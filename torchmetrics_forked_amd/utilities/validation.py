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
import threading
import warnings
from contextlib import contextmanager
from typing import Any, Callable, Dict, Iterator, List, Optional, Tuple, Type

import torch
from torch import Tensor


_ENV_DATA = getattr(os.environ, "_data", None)  # CPython's backing dict: one plain lookup, kept in sync by os.environ[...]
_encodekey = getattr(os.environ, "encodekey", None)  # the key type the backing dict uses (bytes on POSIX, str on Windows)
_ENV_KEY = _encodekey("TMX_VALIDATION") if _ENV_DATA is not None and _encodekey is not None else "TMX_VALIDATION"
if _ENV_DATA is not None and _encodekey is None:
    _ENV_DATA = None


def validation_mode() -> str:
    """``TMX_VALIDATION`` (read on every update: the sink choice follows runtime changes of the variable)."""
    if _ENV_DATA is not None:
        v = _ENV_DATA.get(_ENV_KEY)
        if v is None:
            return "auto"
        return os.fsdecode(v) if isinstance(v, bytes) else v
    return os.environ.get("TMX_VALIDATION", "auto")


# ---------------------------------------------------------------------------------------------------------
# one host read per compute()
# ---------------------------------------------------------------------------------------------------------
class HostCheckBatch:
    """Device-side flags whose host-side consequences (raise / warn) wait for ONE device->host read.

    ``compute()`` used to stall the stream once per check: the deferred input flags, the degenerate-class warnings,
    the NaN-class warning of macro averages ...  Inside :func:`host_checks` each of them only registers its flags
    here (no sync); when the outermost block ends, every flag travels in one small copy and the callbacks run:
    error callbacks first (the first to raise wins, as the eager order would have it), then warning callbacks.
    A ``MetricCollection.compute`` opens the outer block, so a whole collection pays one read."""

    def __init__(self) -> None:
        # (flag tensors, callback over their concatenated values, is-error, consume: zero the flags once read)
        self._items: List[Tuple[List[Tensor], Callable[[List[int]], None], bool, bool]] = []
        self._on_error: List[Callable[[], None]] = []
        self._on_abandon: List[Callable[[], None]] = []

    def add(self, flags: Tensor, callback: Callable[[List[int]], None], error: bool = False) -> None:
        self._items.append(([flags], callback, error, False))

    def add_many(self, flags: List[Tensor], callback: Callable[[List[int]], None], error: bool = False, consume: bool = False) -> None:
        """Several flags read together; ``consume`` zeroes them in the same read (DeferredChecks.check)."""
        self._items.append((list(flags), callback, error, consume))

    def on_error(self, fn: Callable[[], None]) -> None:
        """Run ``fn`` if an error callback raises (e.g. drop a cached compute value)."""
        self._on_error.append(fn)

    def on_abandon(self, fn: Callable[[], None]) -> None:
        """Run ``fn`` if the block ends by an exception before resolving."""
        self._on_abandon.append(fn)

    def abandon(self) -> None:
        fns, self._on_abandon = self._on_abandon, []
        self._items, self._on_error = [], []
        for fn in fns:
            fn()

    @staticmethod
    def _read(items: List[Tuple[List[Tensor], Callable[[List[int]], None], bool, bool]]) -> List[int]:
        """Every flag's elements as ints, in order, in ONE device read; consumed flags are zeroed by that read."""
        flat = [(t, consume) for ts, _, _, consume in items for t in ts]
        devs = {t.device for t, _ in flat}
        if len(devs) == 1 and next(iter(devs)).type == "cuda":
            if _native():  # one native gather kernel + one copy into pinned memory (csrc/flags.hip)
                return torch.ops.tmx.gather_flags([t for t, _ in flat], [int(c) for _, c in flat]).tolist()
        vals = torch.cat([t.reshape(-1).to(torch.int32).cpu() for t, _ in flat]).tolist()
        for t, consume in flat:
            if consume:
                t.zero_()
        return vals

    def resolve(self) -> None:
        self._on_abandon = []
        items, self._items = self._items, []
        on_error, self._on_error = self._on_error, []
        in_forward = _in_forward()
        if in_forward and items and all(not err for _, _, err, _ in items) and all(
            t.is_cuda for ts, _, _, _ in items for t in ts
        ):
            # a forward on the GPU does not wait for the device: its warning flags are read with the next read of any
            # block -- a compute, or a forward that reads error flags anyway (errors of a forward batch stay in the
            # metric's deferred flags, see DeferredChecks.check).  Documented deviation: such batch-value warnings
            # (e.g. "no positive samples") surface late, at most _MAX_PENDING forwards after their batch.
            pend = _pending()
            pend.extend(items)
            _drain_inflight(block=False)
            if len(pend) <= _MAX_PENDING:
                return
            items = list(pend)
            pend.clear()
            if _read_async(items):  # gathered into pinned memory behind an event: read at a later resolve
                return
        else:
            _drain_inflight(block=True)
            pend = _pending()
            if pend and (items or not in_forward):  # warnings parked by earlier forwards ride on this block's read
                items = list(pend) + items
                pend.clear()
        if not items:
            return
        vals = self._read(items)
        chunks, off = [], 0
        for ts, _, _, _ in items:
            n = sum(t.numel() for t in ts)
            chunks.append(vals[off : off + n])
            off += n
        try:
            for (_, cb, err, _), v in zip(items, chunks):
                if err:
                    cb(v)
        except Exception:
            for fn in on_error:
                fn()
            raise
        for (_, cb, err, _), v in zip(items, chunks):
            if not err:
                cb(v)


_OPS = None


def _native() -> bool:
    global _OPS
    ops = _OPS
    if ops is None:  # bound once: a function-level import costs ~2 us per call on the compute path
        from torchmetrics_forked_amd import ops

        _OPS = ops
    return ops.load()


_HOST = threading.local()
_MAX_PENDING = 32  # parked forward warning checks before one read flushes them (asynchronously on the GPU)


def _inflight() -> List[Tuple[List[Tuple[List[Tensor], Callable[[List[int]], None], bool, bool]], Tensor, Any]]:
    q = getattr(_HOST, "inflight", None)
    if q is None:
        q = _HOST.inflight = []
    return q


def _read_async(items: List[Tuple[List[Tensor], Callable[[List[int]], None], bool, bool]]) -> bool:
    """Start one gather of the parked forward flags into pinned host memory without waiting for the device (an
    event marks its completion); False when the flags are not all on one GPU with the native library loaded."""
    flat = [(t, consume) for ts, _, _, consume in items for t in ts]
    devs = {t.device for t, _ in flat}
    if not (len(devs) == 1 and next(iter(devs)).type == "cuda" and _native()):
        return False
    host = torch.ops.tmx.gather_flags_async([t for t, _ in flat], [int(c) for _, c in flat])
    ev = torch.cuda.Event()
    ev.record()
    _inflight().append((items, host, ev))
    return True


def _drain_inflight(block: bool) -> None:
    """Run the callbacks of completed asynchronous flag reads (all of them when ``block``), in issue order."""
    q = _inflight()
    while q:
        items, host, ev = q[0]
        if not block:
            if not ev.query():
                return
        else:
            ev.synchronize()
        q.pop(0)
        vals = host.tolist()
        off = 0
        for ts, cb, _, _ in items:
            n = sum(t.numel() for t in ts)
            cb(vals[off : off + n])
            off += n


def _pending() -> List[Tuple[List[Tensor], Callable[[List[int]], None], bool, bool]]:
    p = getattr(_HOST, "pending", None)
    if p is None:
        p = _HOST.pending = []
    return p


def _batch_stack() -> List[HostCheckBatch]:
    st = getattr(_HOST, "stack", None)
    if st is None:
        st = _HOST.stack = []
    return st


@contextmanager
def forward_scope() -> Iterator[None]:
    """Marks a ``forward``: its batch compute's flag checks must snapshot the flags at once (the accumulated flags are
    OR-ed back before the block's single read); a plain ``compute`` lets that read consume them instead (no kernel)."""
    _HOST.forward_depth = getattr(_HOST, "forward_depth", 0) + 1
    try:
        yield
    finally:
        _HOST.forward_depth -= 1


def enter_forward() -> None:
    """forward_scope()'s entry, for callers that use try / finally instead of a context manager."""
    _HOST.forward_depth = getattr(_HOST, "forward_depth", 0) + 1


def leave_forward() -> None:
    _HOST.forward_depth -= 1


def _in_forward() -> bool:
    return getattr(_HOST, "forward_depth", 0) > 0


def current_host_checks() -> Optional[HostCheckBatch]:
    st = _batch_stack()
    return st[0] if st else None


@contextmanager
def host_checks() -> Iterator[HostCheckBatch]:
    """Collect host checks until the OUTERMOST block ends, then resolve them with a single device->host read."""
    st = _batch_stack()
    if st:
        yield st[0]
        return
    batch = HostCheckBatch()
    st.append(batch)
    ok = False
    try:
        yield batch
        ok = True
    finally:
        st.pop()
        if ok:
            batch.resolve()
        else:
            batch.abandon()


def defer_host_check(flags: Tensor, callback: Callable[[List[int]], None], error: bool = False) -> None:
    """Register ``flags`` with the active :func:`host_checks` block, or read them now when there is none."""
    batch = current_host_checks()
    if batch is None:
        callback(flags.reshape(-1).to(torch.int32).tolist())
    else:
        batch.add(flags, callback, error)


class DeferredChecks:
    """Accumulates device-side failure flags keyed by (exception type, message).

    Two ways to contribute: ``add(bad, ...)`` ORs a boolean tensor in (one small reduction kernel), or
    ``flag(...)`` hands out a persistent ``int32[1]`` device word that native kernels OR into directly while
    they stream the data anyway (zero extra kernels per update).
    """

    def __init__(self) -> None:
        self._flags: Dict[Tuple[Type[Exception], str], Tensor] = {}
        self._held = 0  # > 0 inside a GPU forward that keeps its accumulated flags in place (take_for_forward)

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
        """Raise / warn for every set flag and clear them.  Inside :func:`host_checks` the flags are snapshotted
        on device and inspected together with the block's other checks (one host read for the whole compute)."""
        if not self._flags:
            return
        keys = list(self._flags.keys())
        flags = [self._flags[k] for k in keys]
        warn_keys = [k for k in keys if issubclass(k[0], Warning)]

        def _raise(vals: List[int]) -> None:
            for k, f in zip(keys, vals):
                if f and not issubclass(k[0], Warning):
                    raise k[0](k[1])

        def _warn(vals: List[int]) -> None:
            for k, f in zip(keys, vals):
                if f and issubclass(k[0], Warning):  # deferred warnings (e.g. aggregation nan_strategy="warn")
                    warnings.warn(k[1], k[0], stacklevel=3)

        batch = current_host_checks()
        if batch is None:
            vals = HostCheckBatch._read([(flags, _raise, True, True)])  # one host sync; the flags are cleared
            _warn(vals)
            _raise(vals)
            return
        devs = {f.device for f in flags}
        if _in_forward() and len(devs) == 1 and flags[0].is_cuda:
            # forward on the GPU: no host read now -- the batch's error flags stay set; the forward ORs the accumulated
            # flags back and the next compute() raises (the update-time deferral, extended to forward's batch value)
            return
        if not _in_forward() and len(devs) == 1 and flags[0].is_cuda and _native():
            # compute(): the block's single read returns these flags and clears them (no snapshot kernel; an abandoned
            # block -- an exception before the read -- leaves them set, so the next compute still raises).  Each flag
            # is registered once: the warnings reuse the values the error callback received (registering the flags a
            # second time would let the consuming read clear them before the warning read sees them)
            if not warn_keys:
                batch.add_many(flags, _raise, error=True, consume=True)
                return
            seen: List[List[int]] = []

            def _raise_keep(vals: List[int]) -> None:
                seen.append(vals)
                _raise(vals)

            batch.add_many(flags, _raise_keep, error=True, consume=True)
            batch.add_many([], lambda _v: _warn(seen[0]) if seen else None, error=False)
            return
        # forward(): snapshot + clear on the device now (one native kernel for all flags) -- the forward ORs the
        # accumulated flags back before the block's read, and they must not leak into this batch's check
        if len(devs) == 1 and flags[0].is_cuda and _native():
            snap = torch.ops.tmx.gather_flags_device(flags, [1] * len(flags))
        else:
            snap = torch.cat([f.reshape(-1).to(torch.int32) for f in flags])
            snap = snap.cpu() if len(devs) > 1 else snap
            for f in flags:
                f.zero_()
        batch.add(snap, _raise, error=True)
        if warn_keys:
            batch.add(snap, _warn, error=False)

        def _put_back() -> None:  # the block raised before reading: the flags still owe their exception
            off = 0
            for f in flags:
                n = f.numel()
                f.bitwise_or_(snap[off : off + n].to(f.device, f.dtype).reshape(f.shape))
                off += n

        batch.on_abandon(_put_back)

    def clear(self) -> None:
        if getattr(self, "_held", 0) > 0 and _in_forward():
            # a GPU forward's internal reset(): the accumulated flags stay where they are (nothing was parked), the
            # batch's own flags join them -- both are owed to the next compute()
            return
        for f in self._flags.values():
            f.zero_()

    def snapshot(self) -> Dict[Tuple[Type[Exception], str], Tensor]:
        """Device copies of the current flags (no host sync) — ``forward`` keeps the accumulated ones across its
        internal reset/compute of the batch."""
        return {k: f.clone() for k, f in self._flags.items()}

    def restore(self, snap: Dict[Tuple[Type[Exception], str], Tensor]) -> None:
        """OR previously snapshotted flags back in."""
        for k, f in snap.items():
            cur = self._flags.get(k)
            if cur is None or cur.device != f.device:
                self._flags[k] = f
            else:
                cur.bitwise_or_(f)

    def take(self) -> Optional[Tuple[List[Tuple[Type[Exception], str]], Tensor]]:
        """Snapshot AND clear every flag in one launch (GPU flags; ``snapshot()`` + ``clear()`` otherwise): what
        ``forward`` parks while its batch compute checks only the batch's own flags.  ``give_back`` ORs it in again."""
        if not self._flags:
            return None
        keys = list(self._flags.keys())
        flags = [self._flags[k] for k in keys]
        if len({f.device for f in flags}) == 1 and flags[0].is_cuda and all(f.is_contiguous() for f in flags) and _native():
            return keys, torch.ops.tmx.gather_flags_device(flags, [1] * len(flags))
        snap = self.snapshot()
        self.clear()
        return keys, snap  # type: ignore[return-value]

    def take_for_forward(self) -> Optional[Tuple[List[Tuple[Type[Exception], str]], Tensor]]:
        """``take()`` as ``forward`` needs it: a GPU forward's batch compute never reads device flags (``check``
        returns at once under :func:`forward_scope`), so there is nothing to park -- no snapshot and no OR-back
        launch (2 x 2 launches per forward of a two-metric collection).  Elsewhere: ``take()``."""
        if not self._flags:
            return None
        if _in_forward() and _native():
            flags = list(self._flags.values())
            dev = flags[0].device
            if dev.type == "cuda" and all(f.device == dev for f in flags):
                # nothing is parked, so the forward's internal reset() must not clear them either: hold until give_back
                self._held = getattr(self, "_held", 0) + 1
                return _HOLD  # type: ignore[return-value]
        return self.take()

    def give_back(self, taken: Optional[Tuple[List[Tuple[Type[Exception], str]], Any]]) -> None:
        if taken is None:
            return
        if taken is _HOLD:
            self._held = max(0, getattr(self, "_held", 0) - 1)
            return
        keys, snap = taken
        if isinstance(snap, dict):
            self.restore(snap)
            return
        cur = [self._flags.get(k) for k in keys]
        if all(c is not None and c.device == snap.device and c.is_contiguous() for c in cur) and _native():
            torch.ops.tmx.or_flags(cur, snap)
            return
        off = 0
        for k, c in zip(keys, cur):  # the flag set changed meanwhile (a new device): per-flag restore
            n = 1 if c is None else c.numel()
            piece = snap[off : off + n]
            off += n
            if c is None or c.device != snap.device:
                self._flags[k] = piece.clone()
            else:
                c.bitwise_or_(piece.to(c.dtype).reshape(c.shape))


_HOLD = ("held",)  # take_for_forward's token: flags kept in place (and reset() does not clear them) until give_back


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
