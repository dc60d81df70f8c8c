"""Precision-recall-curve modules and the shared curve-state machinery (API parity: reference
``classification/precision_recall_curve.py:55-675``).

State layout (``thresholds=None``):
  * ``score_hist`` — exact ``int64 [C, 2, 16384]`` histogram for bf16/fp16 scores, ``"sum"``-reduced (RCCL
    all-reduce, sent as int32 whenever that is provably exact), materialised lazily on the first 16-bit batch so fp32 users pay nothing;
  * ``preds`` / ``target`` — ``cat`` lists (reference layout) for fp32/fp64 scores.
With ``thresholds`` given the state is the reference's ``confmat [T, (C,) 2, 2]``.
"""
import os
from typing import Any, List, Optional, Sequence, Tuple, Type, Union

import torch
import torch.distributed as dist
from torch import Tensor
from typing_extensions import Literal

from torchmetrics_forked_amd.classification.base import _ClassificationTaskWrapper
from torchmetrics_forked_amd.functional.classification import _curve_engine as eng
from torchmetrics_forked_amd.functional.classification.precision_recall_curve import (
    BINARY_TARGET_MSG,
    _rows_mc,
    TARGET_RANGE_MSG,
    CurveState,
    _adjust_threshold_arg,
    _binary_precision_recall_curve_arg_validation,
    _binary_precision_recall_curve_tensor_validation,
    _multiclass_precision_recall_curve_arg_validation,
    _multiclass_precision_recall_curve_tensor_validation,
    _multilabel_precision_recall_curve_arg_validation,
    _multilabel_precision_recall_curve_tensor_validation,
    binary_curve_update,
    multiclass_curve_update,
    multilabel_curve_update,
    precision_recall_curve_compute,
)
from torchmetrics_forked_amd.metric import Metric
from torchmetrics_forked_amd.parallel.sync import _collective, sync_states
from torchmetrics_forked_amd.utilities.distributed import gather_all_tensors
from torchmetrics_forked_amd import ops
from torchmetrics_forked_amd.ops import classification as cls_ops
from torchmetrics_forked_amd.utilities.data import dim_zero_cat, dim_zero_sum
from torchmetrics_forked_amd.utilities.validation import validation_mode
from torchmetrics_forked_amd.utilities.enums import ClassificationTask
from torchmetrics_forked_amd.utilities.plot import _AX_TYPE, _PLOT_OUT_TYPE, plot_curve


_SYNC_FREE = os.environ.get("TMX_CURVE_SYNC_FREE", "0") not in ("", "0")
# update lanes (multiclass exact histogram on the GPU, see _CurveMetric._lane_update): on unless TMX_CURVE_LANES=0
_LANES_ON = os.environ.get("TMX_CURVE_LANES", "1") != "0"
_LANE_MIN_ELEMS = 1 << 22  # smaller batches: stream hand-offs cost more than the overlap gains
# the small-class route (C <= 256: one-lane / few-lane rows, csrc/classification.hip) gains nothing from the lanes and
# pays their host hand-offs: C = 10 x 1M 0.060 vs 0.040 ms, C = 64 x 1M 0.161 vs 0.149 (gpurun r7l, tools/gpu_r7f.sh)
_LANE_MIN_CLASSES = 257
_LANE_MAX_HIST_BYTES = 4 << 30  # the second lane's histogram (2 C 16384 int64) is allocated only up to this size


class _Lanes:
    """Two side streams and the second lane's private exact-histogram state (histogram, code range, speculation word).
    ``base``: the histogram lane 0 writes (the metric's ``score_hist``); ``dirty``: lane 1 holds counts not yet
    drained into it; ``busy``: work was issued since the last join."""

    __slots__ = ("streams", "hist", "rng", "mode", "next", "dirty", "busy", "base")

    def __init__(self, hist: Tensor, mode0: Tensor) -> None:
        dev = hist.device
        self.streams = (torch.cuda.Stream(dev), torch.cuda.Stream(dev))
        self.hist = torch.zeros_like(hist)
        self.rng = torch.full((hist.shape[0], 2), -1, dtype=torch.int32, device=dev)
        self.rng[:, 0].fill_(eng.N_CODES)
        self.mode = mode0.clone()  # lane 1 speculates from lane 0's word (a wrong guess only costs a refit)
        for t in (self.hist, self.rng, self.mode):  # issued on lane 1's stream: the allocator must know
            t.record_stream(self.streams[1])
        self.next = 0
        self.dirty = False
        self.busy = False
        self.base: Optional[Tensor] = None

    def bind(self, t: Tensor, k: int) -> None:
        """Tell the caching allocator that lane ``k``'s stream uses ``t`` (its block is not reused before that work)."""
        t.record_stream(self.streams[k])


def _cat_for_read(x: Union[Tensor, List[Tensor]]) -> Tensor:
    """``dim_zero_cat`` for the read-only compute paths: a single-update list state is returned as is (the cat of one
    16.7M-sample fp32 + int64 batch was a 200 MB copy, ~66 us of the compute)."""
    if isinstance(x, list) and len(x) == 1 and x[0].ndim >= 1:
        return x[0]
    return dim_zero_cat(x)


class _CurveMetric(Metric):
    """Owns the curve states; subclasses choose the task and implement ``compute`` from ``_curve_state()``."""

    _task: str = "binary"
    is_differentiable: bool = False
    higher_is_better: Optional[bool] = None
    full_state_update: bool = False

    def _init_curve_states(self, num: int, thresholds: Optional[Union[int, List[float], Tensor]]) -> None:
        self._num = num
        self._hist_dtype: Optional[torch.dtype] = None
        thresholds = _adjust_threshold_arg(thresholds)
        if thresholds is None:
            self.thresholds = thresholds
            self.add_state("preds", default=[], dist_reduce_fx="cat")
            self.add_state("target", default=[], dist_reduce_fx="cat")
            self.add_state("score_hist", default=torch.zeros(0, dtype=torch.long), dist_reduce_fx="sum")
        else:
            self.register_buffer("thresholds", thresholds, persistent=False)
            shape = (len(thresholds), 2, 2) if self._task == "binary" else (len(thresholds), num, 2, 2)
            self.add_state("confmat", default=torch.zeros(*shape, dtype=torch.long), dist_reduce_fx="sum")

    # -------------------------------------------------------------------------------------------- update
    def _kernel_validates(self, preds: Tensor, target: Tensor) -> bool:
        """True when this batch takes a native pass that checks the target values itself (binned or exact
        histogram on the GPU): validation then skips its value-check kernels and hands over a device flag."""
        return ops.use_native(target) and (
            (self.thresholds is not None and self.confmat.dtype == torch.long)
            or (self.thresholds is None and self._hist_ok(preds))
            or (self._task == "multiclass" and self._colmajor_ok(preds) and not (isinstance(self.score_hist, Tensor) and self.score_hist.numel() > 0))
            or self._binary_samples_ok(preds, target)
        )

    def _binary_samples_ok(self, preds: Tensor, target: Tensor) -> bool:
        """GPU fp32 / fp64 binary samples without ignore_index: one native format pass (target check + sigmoid
        decision + copy, csrc/binary_samples.hip) instead of the ATen chain."""
        return (
            self._task == "binary"
            and self.thresholds is None
            and self.ignore_index is None
            and preds.is_cuda
            and preds.dtype in (torch.float32, torch.float64)
            and not target.is_floating_point()
            and not target.is_complex()
            and ops.use_native(preds)
            and not (isinstance(self.score_hist, Tensor) and self.score_hist.numel() > 0)
        )

    def _hist_ok(self, preds: Tensor) -> bool:
        if preds.dtype not in eng.HIST_DTYPES:
            return False
        if self._hist_dtype is None or self._hist_dtype == preds.dtype or self.score_hist.numel() == 0:
            return not (isinstance(self.preds, list) and len(self.preds) > 0)
        return False

    def _mode_state(self, preds: Tensor) -> Optional[Tensor]:
        """Persistent int32[8] device word of the GPU kernels: the speculated softmax decision and the verdict of the
        last batch ([0:2]), the rare-row list counts and the class pass's completion ticket ([2:5]) — see
        curve_hist_kernels.h."""
        if not preds.is_cuda:
            return None
        st = getattr(self, "_spec_mode", None)
        if st is None or st.device != preds.device:
            st = torch.zeros(8, dtype=torch.int32, device=preds.device)
            # seed the first batch's speculation with a range probe (one small kernel, first update only): a wrong
            # first guess costs the class pass a strided refit of every class (~0.7 ms at 65536 x 1000)
            st[0:1].copy_(cls_ops.range_flag(preds))
            self._spec_mode = st
        return st

    def _fresh_hist(self, device: torch.device) -> Tuple[Tensor, Tensor]:
        """A zeroed ``[C, 2, 16384]`` histogram and its empty per-class code range ([16384, -1] rows), built with fill
        kernels only (no host-to-device copy, so no stream synchronisation)."""
        hist = torch.zeros(self._num, 2, eng.N_CODES, dtype=torch.long, device=device)
        rng = torch.full((self._num, 2), -1, dtype=torch.int32, device=device)
        rng[:, 0].fill_(eng.N_CODES)
        return hist, rng

    def _ensure_hist(self, device: torch.device) -> Tensor:
        if self.score_hist.numel() == 0:
            spare = self.__dict__.pop("_hist_spare", None)
            hist, rng = spare if spare is not None and spare[0].device == device else self._fresh_hist(device)
            self.score_hist = hist
            self._set_range(hist, rng)
        return self.score_hist

    def reset(self) -> None:
        """Reference semantics (every state back to its default; ``score_hist`` empty again).  A histogram that was
        in use on the GPU is re-armed as a private spare: its storage goes back to the caching allocator and a zeroed
        one of the same shape is prepared now, so the next epoch's first update binds it instead of allocating and
        zero-filling ``2 C 16384`` int64 (262 MB at C = 1000) inside its own window.  The spare is not state: it is
        dropped from pickles / checkpoints, and a batch on another device ignores it."""
        prev = self.score_hist if self.thresholds is None else None
        rearm = isinstance(prev, Tensor) and prev.numel() > 0 and prev.is_cuda
        dev = prev.device if rearm else None
        prev = None
        super().reset()
        self._invalidate_range()
        self.__dict__.pop("_hist_spare", None)
        if rearm:
            self._hist_spare = self._fresh_hist(dev)

    # ---- occupied code range of ``score_hist`` ------------------------------------------------------------
    # ``_code_range`` (int32[C, 2] = per-class [lo, hi], on the histogram's device) is widened by the class-pass kernel
    # of every update; ``compute`` reads only each class's [lo, hi] and the histogram collectives only the union
    # (softmax scores fill a few binades, about a fifth of the 16384 codes).  It belongs to the tensor object in ``_range_hist``: when ``score_hist`` is
    # replaced by anything that does not maintain it (load_state_dict, forward's merge, .to(...)), the range is
    # recomputed on device from the histogram at its next use — one pass, no host sync.  ``score_hist`` is internal
    # state; code that edits it in place must call ``_invalidate_range()``.
    _range_hist: Optional[Tensor] = None
    _code_range: Optional[Tensor] = None
    _rows_bound: Optional[int] = None  # rows counted into the tracked histogram: bounds every bin (host int)

    def _set_range(self, hist: Tensor, rng: Tensor, rows: Optional[int] = 0) -> None:
        self._range_hist = hist
        self._code_range = rng
        self._rows_bound = rows

    def _after_graph_capture(self) -> None:
        """``utilities.graphs.GraphedUpdate``: replays do not advance the host row count, so the sync bounds the
        histogram bins with a device max instead (the device-side code range stays exact: kernels widen it)."""
        self._rows_bound = None

    def _invalidate_range(self) -> None:
        self._range_hist = None
        self._code_range = None
        self._rows_bound = None

    def _tracked_range(self) -> Optional[Tensor]:
        """The occupied-code range of the current histogram (a device tensor; recomputed when stale)."""
        hist = self.score_hist
        if not isinstance(hist, Tensor) or hist.numel() == 0:
            return None
        if self._range_hist is hist and self._code_range is not None and self._code_range.device == hist.device:
            return self._code_range
        occ = hist.amax(dim=1) > 0  # [C, K]
        idx = torch.arange(hist.shape[-1], device=hist.device)
        rng = torch.stack([torch.where(occ, idx, hist.shape[-1]).amin(-1), torch.where(occ, idx, -1).amax(-1)], 1)
        rng = rng.to(torch.int32).contiguous()
        self._set_range(hist, rng, None)
        return rng

    def _curve_update(
        self, preds: Tensor, target: Tensor, confmat_out: Optional[Tensor] = None, err_flag: Optional[Tensor] = None,
        lanes_ok: bool = True,
    ) -> None:
        thr = self.thresholds
        ii = self.ignore_index
        if thr is not None and ops.use_native(target) and self.confmat.dtype == torch.long:
            # straight into the [T, (C,) 2, 2] state, value check folded into the histogram pass
            if self._task == "binary":
                p, t, cm = preds.reshape(-1, 1, 1), target.reshape(-1, 1, 1), self.confmat.view(len(thr), 1, 2, 2)
            elif self._task == "multiclass":
                (p, t), cm = _rows_mc(preds, target, self._num), self.confmat
            else:
                p, t, cm = preds, target, self.confmat
            cls_ops.binned_curve_update(p, t, thr, cm, self._task, ii, err_flag)
            return
        if thr is not None:
            if self._task == "binary":
                st = binary_curve_update(preds, target, thr, ii)
                self.confmat += st[1][:, 0]
            elif self._task == "multiclass":
                self.confmat += multiclass_curve_update(preds, target, self._num, thr, ii)[1]
            else:
                self.confmat += multilabel_curve_update(preds, target, self._num, thr, ii)[1]
            return
        if self._hist_ok(preds):
            hist = self._ensure_hist(preds.device)
            self._hist_dtype = preds.dtype
            rng = self._tracked_range() if hist.is_cuda else None
            batch = self.__dict__.get("_batch_sink")  # forward(): the batch's own histogram beside the accumulated one
            if batch is not None and (not hist.is_cuda or batch[0].device != hist.device):
                raise RuntimeError("forward's batch histogram lives on another device than the accumulated one")
            if self._task == "binary":
                cls_ops.curve_hist_update(
                    preds.reshape(-1, 1, 1), target.reshape(-1, 1, 1), hist, "binary", ii, err_flag=err_flag, code_range=rng,
                    batch=batch,
                )
            elif self._task == "multiclass":
                # [N, C] inputs (the common case) go through as they are: no movedim / reshape views per update
                p = preds if preds.ndim == 2 else torch.movedim(preds, 1, -1).reshape(-1, self._num)
                t = target if target.ndim == 1 else target.reshape(-1)
                lanes = self._lanes_for(p, hist, rng, batch, lanes_ok)
                if lanes is not None:
                    self._lane_update(lanes, p, t, hist, rng, confmat_out, err_flag)
                else:
                    self._join_side_work()  # (lanes in flight: their histogram work lands before this one's)
                    cls_ops.curve_hist_update(
                        p, t, hist, "multiclass", ii, confmat_out, err_flag, self._mode_state(p), code_range=rng, batch=batch,
                    )
            else:
                cls_ops.curve_hist_update(preds, target, hist, "multilabel", ii, err_flag=err_flag, code_range=rng, batch=batch)
            if rng is None:
                self._invalidate_range()
            elif self._rows_bound is not None:
                self._rows_bound += preds.numel() // self._num
            return
        if self.score_hist.numel() > 0:
            raise NotImplementedError(
                "Mixing 16-bit (exact-histogram) and 32/64-bit score batches in one curve metric is not supported;"
                f" got {preds.dtype} after {self._hist_dtype}. Cast the inputs to one dtype."
            )
        if self._binary_samples_ok(preds, target):
            self.preds.append(cls_ops.binary_samples_format(preds, target, err_flag))
            self.target.append(target.reshape(-1))
            return
        if self._task == "multiclass" and self._colmajor_ok(preds):
            # GPU fp32: softmax decision + transpose in one pass; the state keeps the class-major buffer behind a
            # transposed [N, C] view (same shape / values / checkpoint format as the reference's rows)
            p, t = _rows_mc(preds, target, self._num)
            if ii is not None:
                keep = t != ii
                p, t = p[keep], t[keep]
            self.preds.append(cls_ops.softmax_colmajor(p.contiguous(), t, err_flag).t())
            self.target.append(t)
            return
        if self._task == "binary":
            st = binary_curve_update(preds, target, None, ii, force_samples=True)
        elif self._task == "multiclass":
            st = multiclass_curve_update(preds, target, self._num, None, ii, force_samples=True)
        else:
            st = multilabel_curve_update(preds, target, self._num, None, ii, force_samples=True)
        self.preds.append(st[1])
        self.target.append(st[2])

    # ---- update lanes: consecutive batches' passes overlap ----------------------------------------------------------
    # A multiclass update is a VALU-bound row pass followed by a memory-bound class pass.  Consecutive updates
    # alternate between two lanes, each on its own HIP stream with its own histogram, code range, speculation word and
    # per-stream scratch, so batch k+1's row pass runs beside batch k's class pass (tools/overlap_probe.py: 89.4 ->
    # 77.5 us per 65536 x 1000 bf16 update).  Neither lane runs on the caller's stream: each waits only for the work
    # queued there before it (the inputs).  Every consumer of the states (compute, sync, reset, forward, state_dict,
    # load_state_dict, pickling, device moves -- ``Metric._join_side_work``) first joins both streams into the current
    # one and drains lane 1's counts into ``score_hist`` (``tmx::curve_hist_drain``, over lane 1's occupied range).
    # ``score_hist`` read directly as an attribute between updates holds lane 0's batches only.
    def _lanes_for(self, p: Tensor, hist: Tensor, rng: Optional[Tensor], batch: Any, lanes_ok: bool) -> Optional[_Lanes]:
        if not (
            _LANES_ON and lanes_ok and batch is None and rng is not None and hist.is_cuda and p.numel() >= _LANE_MIN_ELEMS
            and p.shape[-1] >= _LANE_MIN_CLASSES
            and hist.numel() * 8 <= _LANE_MAX_HIST_BYTES and self._range_hist is hist
            and not torch.cuda.is_current_stream_capturing()
        ):
            return None
        lanes = self.__dict__.get("_lanes")
        if lanes is None or lanes.hist.shape != hist.shape or lanes.hist.device != hist.device:
            self._join_side_work()
            lanes = self.__dict__["_lanes"] = _Lanes(hist, self._mode_state(p))
        if lanes.base is not hist:
            self._join_side_work()  # (drains into the histogram lane 1's counts belong to)
            lanes.base = hist
        return lanes

    def _lane_update(self, lanes: _Lanes, p: Tensor, t: Tensor, hist: Tensor, rng: Tensor, confmat_out: Optional[Tensor],
                     err_flag: Optional[Tensor]) -> None:
        k = lanes.next
        s = lanes.streams[k]
        s.wait_stream(torch.cuda.current_stream(p.device))
        ii = self.ignore_index
        with torch.cuda.stream(s):
            h, r, mode = (hist, rng, self._mode_state(p)) if k == 0 else (lanes.hist, lanes.rng, lanes.mode)
            torch.ops.tmx.curve_hist_update(p, t, h, 0, -1 if ii is None else ii, ii is not None, confmat_out, None, err_flag,
                                            mode, r, None, None)
        p.record_stream(s)
        t.record_stream(s)
        if k == 0:
            lanes.bind(hist, 0)
            lanes.bind(rng, 0)
            lanes.bind(mode, 0)
        for x in (confmat_out, err_flag):
            if x is not None:
                lanes.bind(x, k)
        lanes.next = k ^ 1
        lanes.dirty |= k == 1
        lanes.busy = True
        prev = self.__dict__.get("_side_event")
        if prev is not None and prev != self._join_lanes:
            prev()
        self.__dict__["_side_event"] = self._join_lanes

    def _join_lanes(self) -> None:
        lanes = self.__dict__.get("_lanes")
        if lanes is None or not lanes.busy:
            return
        cur = torch.cuda.current_stream(lanes.hist.device)
        for s in lanes.streams:
            cur.wait_stream(s)
        if lanes.dirty and lanes.base is not None:
            base_rng = self._code_range if self._range_hist is lanes.base else None
            if base_rng is not None:
                torch.ops.tmx.curve_hist_drain(lanes.base, base_rng, lanes.hist, lanes.rng)
            else:  # (not reached: the base's range is tracked while lanes run) -- dense merge, range recomputed
                lanes.base.add_(lanes.hist)
                lanes.hist.zero_()
                lanes.rng[:, 0].fill_(eng.N_CODES)
                lanes.rng[:, 1].fill_(-1)
                if self._range_hist is lanes.base:
                    self._invalidate_range()
        lanes.dirty = False
        lanes.busy = False
        lanes.next = 0

    # ---- steady-state GPU update: one native call ----------------------------------------------------------------
    # After an update took the exact-histogram route on the GPU, the next ones with the same kind of inputs skip the
    # generic plumbing (sink / route / range / mode-word lookups, ~10 us of Python) and call the native op directly.
    # Every cached object is re-validated by identity per call (a reset, load_state_dict, .to(), sync or a forward's
    # batch histogram replaces it and falls back to the full path, which re-arms); the host-side shape / dtype checks
    # of the reference's validation are kept inline, the target value check stays in the kernel (deferred flag).
    # multiclass: [N, C] scores, [N] targets; binary (no ignore_index): scores and targets of one shape.
    def _arm_fast_update(self, preds: Tensor, target: Tensor) -> None:
        hist = self.score_hist if self.thresholds is None else None
        ok = (
            isinstance(hist, Tensor) and hist.is_cuda and hist.numel() > 0 and preds.is_cuda
            and preds.dtype in eng.HIST_DTYPES and self._range_hist is hist and self._code_range is not None
            and self._rows_bound is not None and (not self.validate_args or self._deferred is not None)
        )
        if ok and self._task == "multiclass":
            ok = preds.ndim == 2 and target.ndim == 1 and "_spec_mode" in self.__dict__
        elif ok and self._task == "binary":
            ok = self.ignore_index is None
        else:
            ok = False
        self.__dict__["_fast_update"] = (hist, preds.dtype, preds.get_device()) if ok else None

    def _fast_hist_update(self, preds: Tensor, target: Tensor) -> bool:
        fast = self.__dict__.get("_fast_update")
        if fast is None:
            return False
        hist, dtype, dev = fast
        d = self.__dict__
        if (
            self.score_hist is not hist or d.get("_batch_sink") is not None or self._range_hist is not hist
            or type(preds) is not Tensor or type(target) is not Tensor or preds.dtype is not dtype
            or preds.get_device() != dev or target.get_device() != dev or target.is_floating_point() or self._rows_bound is None
        ):
            return False
        multiclass = self._task == "multiclass"
        if multiclass:
            if preds.ndim != 2 or target.ndim != 1 or preds.shape[0] != target.shape[0] or preds.shape[1] != self._num:
                return False
            if _LANES_ON and preds.numel() >= _LANE_MIN_ELEMS and preds.shape[1] >= _LANE_MIN_CLASSES:
                return False  # the update lanes take it (_lane_update)
        if d.get("_side_event") is not None:
            self._join_side_work()
        elif preds.shape != target.shape:
            return False
        err = None
        if self.validate_args:
            if validation_mode() == "eager":
                return False
            err = self._deferred.flag(RuntimeError, TARGET_RANGE_MSG if multiclass else BINARY_TARGET_MSG, hist.device)
        ii = self.ignore_index
        torch.ops.tmx.curve_hist_update(
            preds, target, hist, 0 if multiclass else 1, -1 if ii is None else ii, ii is not None, None, None, err,
            d["_spec_mode"] if multiclass else None, self._code_range, None, None,
        )
        d["_rows_bound"] = self._rows_bound + (preds.shape[0] if multiclass else preds.numel())
        return True

    # ---- forward on the exact histogram (GPU) -----------------------------------------------------------------------
    # The reference's reduce-state forward parks the global state, resets, updates a fresh state, computes and merges
    # (metric.py:352-390): for a [C, 2, 16384] int64 histogram that is a 262 MB zero-filled allocation plus a dense
    # ``glob + local`` per call at C = 1000.  Here the global histogram is updated in place and the same class pass also
    # flushes the batch's counts into a per-metric scratch histogram (zero outside forward) with its own code range;
    # the batch value is reduced from that scratch over the batch's range, which is then zeroed again.
    def _batch_sink_ok(self) -> bool:
        h = self.score_hist if self.thresholds is None else None
        return isinstance(h, Tensor) and h.numel() > 0 and h.is_cuda and not self.dist_sync_on_step

    def _batch_scratch(self) -> Tuple[Tensor, Tensor]:
        h = self.score_hist
        sc = self.__dict__.get("_batch_bufs")
        if sc is None or sc[0].shape != h.shape or sc[0].device != h.device:
            rng = torch.full((h.shape[0], 2), -1, dtype=torch.int32, device=h.device)
            rng[:, 0].fill_(eng.N_CODES)
            sc = (torch.zeros_like(h), rng)
            self.__dict__["_batch_bufs"] = sc
        return sc

    def _forward_reduce_state_update(self, *args: Any, **kwargs: Any) -> Any:
        if not self._batch_sink_ok():
            return super()._forward_reduce_state_update(*args, **kwargs)
        ctx = self._fused_forward_begin()
        try:
            self.update(*args, **kwargs)
        except BaseException:
            self._fused_forward_abort(ctx)
            raise
        return self._fused_forward_end(ctx)

    def _fused_forward_begin(self) -> Tuple[Any, ...]:
        if not self._batch_sink_ok():
            return super()._fused_forward_begin()
        self._join_side_work()
        snap_def = None
        if self._deferred is not None:
            snap_def = self._deferred.take_for_forward()
        count = self._update_count
        saved = self._enter_batch_mode()
        self.__dict__["_batch_sink"] = self._batch_scratch()
        return ("batch_sink", count, saved, snap_def)

    def _fused_forward_abort(self, ctx: Tuple[Any, ...]) -> None:
        sink = self.__dict__.pop("_batch_sink", None)
        if sink is not None:
            cls_ops.curve_hist_zero(*sink)
        _, count, saved, snap_def = ctx
        self._update_count = count
        self._leave_batch_mode(saved)
        if snap_def is not None:
            self._deferred.give_back(snap_def)

    def _fused_forward_end(self, ctx: Tuple[Any, ...]) -> Any:
        if not (isinstance(ctx, tuple) and ctx and ctx[0] == "batch_sink"):
            return super()._fused_forward_end(ctx)
        _, count, saved, snap_def = ctx
        self.__dict__["_batch_view"] = True
        cleared = self.__dict__["_batch_cleared"] = [False]
        try:
            batch_val = self.compute()
        finally:
            self.__dict__["_batch_view"] = False
            sink = self.__dict__.pop("_batch_sink", None)
            if sink is not None and not cleared[0]:
                cls_ops.curve_hist_zero(*sink)
            self._update_count = count + 1
            self._leave_batch_mode(saved)
            if snap_def is not None:
                self._deferred.give_back(snap_def)
        self._forward_cache = batch_val
        return batch_val

    def _reduce_states(self, incoming_state: dict) -> None:
        """``forward`` merge: the lazily materialised histogram may be empty on either side."""
        if self.thresholds is None:
            glob, local = incoming_state["score_hist"], self.score_hist
            if glob.numel() == 0 or local.numel() == 0:
                merged = local if glob.numel() == 0 else glob
                incoming_state = dict(incoming_state)
                incoming_state["score_hist"] = torch.zeros_like(merged)
                self.score_hist = merged
        super()._reduce_states(incoming_state)

    # ---------------------------------------------------------------------------------------------- sync
    _shard_info: Optional[Tuple[int, int, int, Any]] = None  # (first class, classes owned, shard rows, group)

    def _shardable(self, dist_sync_fn: Any) -> bool:
        return (
            self.sharded_compute
            and self.thresholds is None
            and self._task != "binary"
            and getattr(self, "average", None) != "micro"
            and self.score_hist.numel() > 0
            and (dist_sync_fn is None or dist_sync_fn is gather_all_tensors)
        )

    def _sync_sharded(self, group: Optional[Any], narrow: bool, lo: int, hi: int) -> None:
        """State-parallel sync: reduce-scatter the exact histogram by class so each rank owns
        ``ceil(C / W)`` classes, and sync the remaining states normally.  Only the occupied code range ``[lo, hi]``
        (the same on every rank) travels."""
        world = dist.get_world_size(group)
        rank = dist.get_rank(group)
        c = self._num
        per = -(-c // world)
        sl = self.score_hist[:, :, lo : hi + 1]
        full = sl.to(torch.int32) if narrow else sl.contiguous()
        if per * world != c:
            full = torch.cat([full, full.new_zeros(per * world - c, *full.shape[1:])])
        shard = full.new_empty(per, *full.shape[1:])
        _collective(dist.reduce_scatter_tensor, shard, full.contiguous(), op=dist.ReduceOp.SUM, what="reduce_scatter(score_hist)", group=group)
        others = {k: v for k, v in self.metric_state.items() if k != "score_hist"}
        for name, val in sync_states(others, self._reductions, group=group).items():
            setattr(self, name, val)
        first = rank * per
        owned = max(0, min(per, c - first))
        self.score_hist = hist = self._owned_hist(owned, lo, hi, shard[:owned])
        self._set_range(hist, torch.tensor([lo, hi], dtype=torch.int32, device=hist.device).repeat(owned, 1), None)
        self._shard_info = (first, owned, per, group)

    def _owned_hist(self, owned: int, lo: int, hi: int, window: Tensor, key: str = "_owned_buf", live: Optional[Tensor] = None) -> Tensor:
        """The synced histogram ``[owned, 2, 16384]`` (the owned classes of a sharded sync, every class of a replicated
        one: ``key``) with ``window`` at codes ``[lo, hi]`` and zeros elsewhere, in a buffer kept across syncs: only
        the previous sync's window is cleared (a fresh full-width int64 allocation + fill per sync was 8 MiB per owned
        class group at C = 1000 / 8 ranks, 262 MB per replicated sync).  The buffer is only ever the synced state
        between ``sync`` and ``unsync`` -- ``unsync`` puts the local histogram back -- so reusing it at the next sync
        never touches a live state (a buffer that is still the metric's state is never reused)."""
        dev, k = self.score_hist.device, eng.N_CODES
        held = self.__dict__.get(key)
        live = self.score_hist if live is None else live
        if held is None or held[0].shape[0] != owned or held[0].device != dev or held[0] is live:
            buf = torch.zeros(owned, 2, k, dtype=torch.long, device=dev)
        else:
            buf, plo, phi = held
            buf[:, :, plo : phi + 1].zero_()
        buf[:, :, lo : hi + 1] = window
        self.__dict__[key] = (buf, lo, hi)
        return buf

    def _leave_batch_mode(self, saved_compute_on_cpu: bool) -> None:
        super()._leave_batch_mode(saved_compute_on_cpu)
        self._shard_info = None  # a batch compute's sharded sync is never unsynced: forget it with the synced flag

    def unsync(self, should_unsync: bool = True) -> None:
        super().unsync(should_unsync)
        if should_unsync:
            self._shard_info = None
            saved = getattr(self, "_range_saved", None)
            if saved is not None:
                self._range_hist, self._code_range, self._rows_bound = saved
                self._range_saved = None

    def _sharded_scores(self) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
        """(auroc, ap, P, N) for all classes from this rank's class shard + one small all-gather."""
        first, owned, per, group = self._shard_info  # type: ignore[misc]
        world = dist.get_world_size(group)
        local = torch.zeros(4, per, dtype=torch.float64, device=self.score_hist.device)
        if owned > 0:
            auc, ap, pos, neg = eng.hist_scores(self.score_hist, self._tracked_range())
            local[0, :owned], local[1, :owned] = auc.double(), ap.double()
            local[2, :owned], local[3, :owned] = pos.double(), neg.double()
        backend = dist.get_backend(group) if group is not None else dist.get_backend()
        comm = local if backend == "nccl" or not local.is_cuda else local.cpu()
        allv = comm.new_empty(world, 4, per)
        _collective(dist.all_gather_into_tensor, allv.view(-1), comm.reshape(-1), what="all_gather(per-class scores)", group=group)
        allv = allv.permute(1, 0, 2).reshape(4, world * per)[:, : self._num].to(local.device)
        from torchmetrics_forked_amd.functional.classification.auroc import ExactScores

        summ = cls_ops.curve_summary(allv.t().contiguous()) if allv.is_cuda else None
        return ExactScores.of(allv[0], allv[1], allv[2], allv[3], summ)

    _DTYPE_CODES = {None: 0, torch.bfloat16: 1, torch.float16: 2}

    def _sync_dist(self, dist_sync_fn: Any = None, process_group: Optional[Any] = None) -> None:
        """The exact histogram travels (a) as int32 whenever the summed per-rank bin bounds prove every global
        bin fits (half the bytes) and (b) only over the code range ``[lo, hi]`` some rank occupies: softmax scores
        fill a few bf16 binades, about a fifth of the 16384 codes.  One tiny all-gather of per-rank (has-histogram,
        bin bound, lo, hi, score dtype, has-samples) decides both and checks that the ranks agree on the state kind.
        The bin bound is the number of rows counted (host-tracked); only a histogram of unknown origin (loaded,
        merged) pays a device max over its bins.  Ranks without a histogram adopt the score dtype of the others."""
        if self.thresholds is None and self._sync_free(dist_sync_fn):
            self._sync_dist_free(process_group or self.process_group)
            return
        if self.thresholds is None:
            group = process_group or self.process_group
            backend = dist.get_backend(group) if group is not None else dist.get_backend()
            dev = self.score_hist.device if backend != "nccl" or self.score_hist.is_cuda else torch.device("cuda")
            has = self.score_hist.numel() > 0
            k = eng.N_CODES
            dcode = self._DTYPE_CODES.get(self._hist_dtype if has else None, 0)
            has_samples = int(isinstance(self.preds, list) and len(self.preds) > 0)
            if has:
                rng = self._tracked_range()
                if self._rows_bound is not None:
                    bound = torch.tensor([self._rows_bound], dtype=torch.long, device=rng.device)
                else:
                    bound = self.score_hist.amax().reshape(1)
                stats = torch.cat([
                    torch.ones(1, dtype=torch.long, device=rng.device), bound.long(),
                    rng[:, 0].amin().reshape(1).long(), rng[:, 1].amax().reshape(1).long(),
                    torch.tensor([dcode, has_samples], dtype=torch.long, device=rng.device),
                ])
            else:
                stats = torch.tensor([0, 0, k, -1, 0, has_samples], dtype=torch.long, device=dev)
            stats = stats.to(dev if backend == "nccl" else "cpu")
            allv = torch.empty(dist.get_world_size(group), stats.numel(), dtype=stats.dtype, device=stats.device)
            _collective(dist.all_gather_into_tensor, allv.view(-1), stats, what="all_gather(histogram stats)", group=group)
            allv = allv.tolist()
            used, bound = sum(v[0] for v in allv), sum(v[1] for v in allv)
            lo, hi = min(v[2] for v in allv), max(v[3] for v in allv)
            dcodes = {v[4] for v in allv if v[0]}
            if len(dcodes) > 1:
                raise RuntimeError(
                    "Ranks accumulated curve scores in different 16-bit dtypes (bf16 on some, fp16 on others); their"
                    " exact histograms cannot be combined. Cast the inputs to one dtype on every rank."
                )
            if used and any(v[5] for v in allv):
                raise RuntimeError(
                    "Some ranks hold 16-bit score histograms and others fp32/fp64 score lists for the same curve metric;"
                    " cast the inputs to one dtype on every rank."
                )
            if used and not has:
                self._hist_dtype = {v: kk for kk, v in self._DTYPE_CODES.items()}[dcodes.pop()]
            narrow = used > 0 and bound < 2**31 - 1
            if hi < lo:  # no rank counted anything: keep one bin so the collectives stay well-formed
                lo = hi = 0
            if used and self.score_hist.numel() == 0:
                self._ensure_hist(self.device)
            self._range_saved = (self._range_hist, self._code_range, self._rows_bound)
            if self._shardable(dist_sync_fn):
                self._sync_sharded(group, narrow, lo, hi)
                return
            if used and (dist_sync_fn is None or dist_sync_fn is gather_all_tensors):
                shape = self.score_hist.shape
                local_hist = self.score_hist
                sl = self.score_hist[:, :, lo : hi + 1]
                self.score_hist = sl.to(torch.int32) if narrow else sl.contiguous()
                try:
                    super()._sync_dist(dist_sync_fn, process_group)
                finally:
                    synced = self.score_hist
                    hist = self._owned_hist(shape[0], lo, hi, synced, key="_synced_buf", live=local_hist)
                    self.score_hist = hist
                    self._set_range(hist, torch.tensor([lo, hi], dtype=torch.int32, device=hist.device).repeat(shape[0], 1), bound)
                return
        super()._sync_dist(dist_sync_fn, process_group)

    def _sync_free(self, dist_sync_fn: Any) -> bool:
        """The host-synchronisation-free sync (``_sync_dist_free``): under HIP-graph capture, or when asked for with
        ``TMX_CURVE_SYNC_FREE=1``.  Needs the exact histogram on this rank (16-bit scores) and the default gather."""
        if dist_sync_fn is not None and dist_sync_fn is not gather_all_tensors:
            return False
        if isinstance(self.preds, list) and self.preds:
            return False
        want = _SYNC_FREE or (torch.cuda.is_available() and torch.cuda.is_current_stream_capturing())
        return bool(want) and (self.score_hist.numel() > 0 or self._hist_dtype is not None or _SYNC_FREE)

    def _sync_dist_free(self, group: Optional[Any]) -> None:
        """Sync without a device-to-host read: the collective sizes are fixed by the host alone, so the histogram
        travels over its full code range as int64 (the default sync's narrowing to the occupied range and to int32
        is decided from a gathered per-rank summary, which the host must read); the per-class code ranges are
        combined on the device (one MIN all-reduce of (lo, -hi)).  Every rank must hold 16-bit-score histograms (a
        rank without a batch contributes zeros); the dtype agreement check of the default sync is not made.
        Sharded compute reduce-scatters by class as the default sync does.  (Reference: ``metric.py:423-453``.)"""
        hist = self._ensure_hist(self.device)
        rng = self._tracked_range()
        self._range_saved = (self._range_hist, self._code_range, self._rows_bound)
        packed = torch.stack([rng[:, 0], -rng[:, 1]], 1).contiguous()
        _collective(dist.all_reduce, packed, op=dist.ReduceOp.MIN, what="all_reduce(code ranges)", group=group)
        rng_all = torch.stack([packed[:, 0], -packed[:, 1]], 1)
        if self._shardable(None):
            world = dist.get_world_size(group)
            rank = dist.get_rank(group)
            c = self._num
            per = -(-c // world)
            full = hist if per * world == c else torch.cat([hist, hist.new_zeros(per * world - c, *hist.shape[1:])])
            shard = full.new_empty(per, *full.shape[1:])
            _collective(dist.reduce_scatter_tensor, shard, full.contiguous(), op=dist.ReduceOp.SUM,
                        what="reduce_scatter(score_hist)", group=group)
            self._sync_fixed_states([k for k in self._defaults if k != "score_hist"], group)
            first = rank * per
            owned = max(0, min(per, c - first))
            self.score_hist = shard[:owned]
            self._set_range(self.score_hist, rng_all[first : first + owned].contiguous(), None)
            self._shard_info = (first, owned, per, group)
            return
        self._sync_fixed_states(list(self._defaults), group)
        self._set_range(self.score_hist, rng_all.to(torch.int32).contiguous(), None)

    def _sync_fixed_states(self, names: List[str], group: Optional[Any]) -> None:
        """The sync-free path's remaining states: a sum-reduced tensor (the same shape on every rank) is one in-place
        SUM all-reduce of a copy (the pre-sync value stays in the unsync cache); an empty list state stays empty (the
        sync-free contract: every rank holds histograms, so no rank has list samples).  Anything else goes through the
        generic gather, which may read sizes on the host."""
        rest = {}
        for name in names:
            val = getattr(self, name)
            if isinstance(val, Tensor) and self._reductions[name] is dim_zero_sum:
                out = val.clone()
                _collective(dist.all_reduce, out, op=dist.ReduceOp.SUM, what=f"all_reduce({name})", group=group)
                setattr(self, name, out)
            elif isinstance(val, list) and len(val) == 0:
                continue
            else:
                rest[name] = val
        if rest:
            for name, val in sync_states(rest, self._reductions, group=group).items():
                setattr(self, name, val)

    # ------------------------------------------------------------------------------------------- compute
    def _colmajor_ok(self, preds: Tensor) -> bool:
        return preds.is_cuda and preds.dtype == torch.float32 and self._num <= 1024 and self._num % 4 == 0 and ops.use_native(preds)

    def _curve_state(self, lazy: bool = False) -> CurveState:
        """``lazy=True`` (class-averaged AUROC / AP only): fp32 samples written class-major by the GPU update are
        handed over as ``ColumnChunks`` and streamed in place instead of being concatenated."""
        if self.thresholds is not None:
            cm = self.confmat.unsqueeze(1) if self._task == "binary" else self.confmat
            return ("binned", cm)
        if self.__dict__.get("_batch_view") and self.__dict__.get("_batch_sink") is not None:
            bh, br = self.__dict__["_batch_sink"]
            # (the one-element marker: a consumer that reduces AND clears the scratch sets it -- no zero launches after)
            return ("hist", bh, self._hist_dtype or torch.bfloat16, br, self.__dict__.setdefault("_batch_cleared", [False]))
        if isinstance(self.score_hist, Tensor) and self.score_hist.numel() > 0:
            return ("hist", self.score_hist, self._hist_dtype or torch.bfloat16, self._tracked_range())
        if lazy and isinstance(self.preds, list) and self.preds:
            cols = [p.t() for p in self.preds]
            if all(c.is_cuda and c.dtype == torch.float32 and c.is_contiguous() for c in cols):
                return ("samples", eng.ColumnChunks(cols), dim_zero_cat(self.target))
        return ("samples", _cat_for_read(self.preds), _cat_for_read(self.target))

    def plot(
        self, curve: Optional[Tuple] = None, score: Optional[Union[Tensor, bool]] = None, ax: Optional[_AX_TYPE] = None
    ) -> _PLOT_OUT_TYPE:
        curve_computed = curve or self.compute()
        if isinstance(curve_computed, Tensor):
            return self._plot(curve_computed, ax)
        score = self._auc_for_plot(curve_computed) if isinstance(score, bool) and score else score
        return plot_curve(curve_computed, score=score, ax=ax, label_names=self._label_names, name=self.__class__.__name__)

    _label_names = ("Recall", "Precision")

    def _auc_for_plot(self, curve: Tuple) -> Optional[Tensor]:
        from torchmetrics_forked_amd.utilities.compute import _auc_compute_without_check

        x, y = curve[1], curve[0]
        if isinstance(x, Tensor) and x.ndim == 1:
            return _auc_compute_without_check(x, y, -1.0)
        return torch.stack([_auc_compute_without_check(a, b, -1.0) for a, b in zip(x, y)])


class BinaryPrecisionRecallCurve(_CurveMetric):
    """Precision-recall curve for binary tasks.

    Example:
        >>> import torch
        >>> from torchmetrics_forked_amd.classification import BinaryPrecisionRecallCurve
        >>> precision, recall, thresholds = BinaryPrecisionRecallCurve()(torch.tensor([0.0, 0.5, 0.7, 0.8]), torch.tensor([0, 1, 1, 0]))
        >>> precision
        tensor([0.5000, 0.6667, 0.5000, 0.0000, 1.0000])
        >>> recall
        tensor([1.0000, 1.0000, 0.5000, 0.0000, 0.0000])
    """

    _task = "binary"

    def __init__(
        self,
        thresholds: Optional[Union[int, List[float], Tensor]] = None,
        ignore_index: Optional[int] = None,
        validate_args: bool = True,
        **kwargs: Any,
    ) -> None:
        super().__init__(**kwargs)
        if validate_args:
            _binary_precision_recall_curve_arg_validation(thresholds, ignore_index)
        self.ignore_index = ignore_index
        self.validate_args = validate_args
        self._init_curve_states(1, thresholds)

    def update(self, preds: Tensor, target: Tensor) -> None:
        if self._fast_hist_update(preds, target):
            return
        err = None
        if self.validate_args:
            sink = self._validation_sink(target)
            in_kernel = sink is not None and self._kernel_validates(preds, target)
            _binary_precision_recall_curve_tensor_validation(preds, target, self.ignore_index, sink, check_values=not in_kernel)
            err = sink.flag(RuntimeError, BINARY_TARGET_MSG, target.device) if in_kernel else None
        self._curve_update(preds, target, err_flag=err)
        self._arm_fast_update(preds, target)

    def compute(self) -> Tuple[Tensor, Tensor, Tensor]:
        return precision_recall_curve_compute(self._curve_state(), "binary", 1, self.thresholds)


class MulticlassPrecisionRecallCurve(_CurveMetric):
    """One-vs-rest precision-recall curves for multiclass tasks."""

    _task = "multiclass"

    def __init__(
        self,
        num_classes: int,
        thresholds: Optional[Union[int, List[float], Tensor]] = None,
        average: Optional[Literal["micro", "macro"]] = None,
        ignore_index: Optional[int] = None,
        validate_args: bool = True,
        **kwargs: Any,
    ) -> None:
        super().__init__(**kwargs)
        if validate_args:
            _multiclass_precision_recall_curve_arg_validation(num_classes, thresholds, ignore_index, average)
        self.num_classes = num_classes
        self.average = average
        self.ignore_index = ignore_index
        self.validate_args = validate_args
        self._init_curve_states(num_classes, thresholds)

    def _fusion_key(self) -> Optional[Tuple]:
        """Key under which a ``MetricCollection`` may fuse this update with others (see ``ops.fused``)."""
        if self.thresholds is not None:
            return None
        return ("multiclass_scores", self.num_classes, self.ignore_index)

    def _validate_fused(self, preds: Tensor, target: Tensor) -> Optional[Tensor]:
        """Validate; on the GPU exact-histogram path the target range check is done inside the HIP kernel.

        Returns the device error flag the kernel must OR into (or ``None``)."""
        if not self.validate_args:
            return None
        sink = self._validation_sink(target)
        in_kernel = sink is not None and self._kernel_validates(preds, target)
        _multiclass_precision_recall_curve_tensor_validation(
            preds, target, self.num_classes, self.ignore_index, sink, check_values=not in_kernel
        )
        return sink.flag(RuntimeError, TARGET_RANGE_MSG, target.device) if in_kernel else None

    def update(self, preds: Tensor, target: Tensor) -> None:
        if self._fast_hist_update(preds, target):
            return
        err = self._validate_fused(preds, target)
        self._curve_update(preds, target, err_flag=err)
        self._arm_fast_update(preds, target)

    def compute(self) -> Union[Tuple[Tensor, Tensor, Tensor], Tuple[List[Tensor], List[Tensor], List[Tensor]]]:
        return precision_recall_curve_compute(
            self._curve_state(), "multiclass", self.num_classes, self.thresholds, self.ignore_index, self.average
        )


class MultilabelPrecisionRecallCurve(_CurveMetric):
    """Per-label precision-recall curves."""

    _task = "multilabel"

    def __init__(
        self,
        num_labels: int,
        thresholds: Optional[Union[int, List[float], Tensor]] = None,
        ignore_index: Optional[int] = None,
        validate_args: bool = True,
        **kwargs: Any,
    ) -> None:
        super().__init__(**kwargs)
        if validate_args:
            _multilabel_precision_recall_curve_arg_validation(num_labels, thresholds, ignore_index)
        self.num_labels = num_labels
        self.ignore_index = ignore_index
        self.validate_args = validate_args
        self._init_curve_states(num_labels, thresholds)

    def update(self, preds: Tensor, target: Tensor) -> None:
        err = None
        if self.validate_args:
            sink = self._validation_sink(target)
            in_kernel = sink is not None and self._kernel_validates(preds, target)
            _multilabel_precision_recall_curve_tensor_validation(
                preds, target, self.num_labels, self.ignore_index, sink, check_values=not in_kernel
            )
            err = sink.flag(RuntimeError, BINARY_TARGET_MSG, target.device) if in_kernel else None
        self._curve_update(preds, target, err_flag=err)

    def compute(self) -> Union[Tuple[Tensor, Tensor, Tensor], Tuple[List[Tensor], List[Tensor], List[Tensor]]]:
        return precision_recall_curve_compute(
            self._curve_state(), "multilabel", self.num_labels, self.thresholds, self.ignore_index
        )


def _curve_task_factory(
    task: str,
    binary_cls: Type[Metric],
    multiclass_cls: Type[Metric],
    multilabel_cls: Type[Metric],
    binary_args: tuple,
    multiclass_args: tuple,
    multilabel_args: tuple,
    num_classes: Optional[int],
    num_labels: Optional[int],
    kwargs: dict,
) -> Metric:
    task = ClassificationTask.from_str(task)
    if task == ClassificationTask.BINARY:
        return binary_cls(*binary_args, **kwargs)
    if task == ClassificationTask.MULTICLASS:
        if not isinstance(num_classes, int):
            raise ValueError(f"`num_classes` is expected to be `int` but `{type(num_classes)} was passed.`")
        return multiclass_cls(*multiclass_args, **kwargs)
    if task == ClassificationTask.MULTILABEL:
        if not isinstance(num_labels, int):
            raise ValueError(f"`num_labels` is expected to be `int` but `{type(num_labels)} was passed.`")
        return multilabel_cls(*multilabel_args, **kwargs)
    raise ValueError(f"Task {task} not supported!")


class PrecisionRecallCurve(_ClassificationTaskWrapper):
    """Task wrapper returning Binary/Multiclass/MultilabelPrecisionRecallCurve."""

    def __new__(  # type: ignore[misc]
        cls: Type["PrecisionRecallCurve"],
        task: Literal["binary", "multiclass", "multilabel"],
        thresholds: Optional[Union[int, List[float], Tensor]] = None,
        num_classes: Optional[int] = None,
        num_labels: Optional[int] = None,
        ignore_index: Optional[int] = None,
        validate_args: bool = True,
        **kwargs: Any,
    ) -> Metric:
        kwargs.update({"thresholds": thresholds, "ignore_index": ignore_index, "validate_args": validate_args})
        return _curve_task_factory(
            task, BinaryPrecisionRecallCurve, MulticlassPrecisionRecallCurve, MultilabelPrecisionRecallCurve,
            (), (num_classes,), (num_labels,), num_classes, num_labels, kwargs,
        )
