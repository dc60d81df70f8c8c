"""Stat-scores modules (API parity: reference ``classification/stat_scores.py:43-546``).

Global states are ``int64`` tensors reduced with ``"sum"`` (one coalesced RCCL all-reduce for all four);
``samplewise`` states are ``cat`` lists.  Updates run one fused HIP pass per batch (see functional module).
"""
from typing import Any, Callable, Dict, List, Optional, Sequence, Tuple, Type, Union

import torch
from torch import Tensor
from typing_extensions import Literal

from torchmetrics_forked_amd import ops
from torchmetrics_forked_amd.classification.base import _ClassificationTaskWrapper
from torchmetrics_forked_amd.functional.classification.stat_scores import (
    _binary_stat_scores_arg_validation,
    _binary_stat_scores_compute,
    _binary_stat_scores_format,
    _binary_stat_scores_tensor_validation,
    _binary_stat_scores_update,
    _binary_stats_fused,
    _binary_value_flags,
    _multiclass_pairs_view,
    _multiclass_range_flags,
    _multiclass_stat_scores_accumulate,
    _multiclass_stat_scores_arg_validation,
    _multiclass_stat_scores_compute,
    _multiclass_stat_scores_tensor_validation,
    _multiclass_stat_scores_update,
    _multilabel_stat_scores_arg_validation,
    _multilabel_stat_scores_compute,
    _multilabel_stat_scores_format,
    _multilabel_stat_scores_tensor_validation,
    _multilabel_stat_scores_update,
    _multilabel_stats_fused,
)
from torchmetrics_forked_amd.metric import Metric
from torchmetrics_forked_amd.ops import classification as cls_ops
from torchmetrics_forked_amd.utilities.data import dim_zero_cat
from torchmetrics_forked_amd.utilities.enums import ClassificationTask
from torchmetrics_forked_amd.utilities.plot import _AX_TYPE, _PLOT_OUT_TYPE


class _AbstractStatScores(Metric):
    tp: Union[List[Tensor], Tensor]
    fp: Union[List[Tensor], Tensor]
    tn: Union[List[Tensor], Tensor]
    fn: Union[List[Tensor], Tensor]

    def _create_state(self, size: int, multidim_average: str = "global") -> None:
        for name in ("tp", "fp", "tn", "fn"):
            if multidim_average == "samplewise":
                self.add_state(name, [], dist_reduce_fx="cat")
            else:
                self.add_state(name, torch.zeros(size, dtype=torch.long), dist_reduce_fx="sum")

    def _int64_states(self) -> bool:
        """The native kernels count into int64 states; after ``set_dtype`` (which, as in the reference, casts every
        state) the generic update path takes over."""
        d = self.__dict__
        for n in ("tp", "fp", "tn", "fn"):
            v = d.get(n)
            if not isinstance(v, Tensor) or v.dtype != torch.long:
                return False
        return True

    def _scratch(self, numel: int, device: torch.device) -> Tensor:
        """Zero int64 scratch of the fused GPU kernels (left at zero by every launch; not a metric state)."""
        buf = getattr(self, "_ticket", None)
        if buf is None or buf.device != device or buf.numel() < numel:
            buf = self._ticket = torch.zeros(numel, dtype=torch.long, device=device)
        return buf

    def _binary_fused_update(self, preds: Tensor, target: Tensor, num_labels: int, validate: Callable) -> bool:
        """GPU fast path for global binary / multilabel stats: one kernel, counts straight into the states, value
        checks as device flags (csrc/classification.hip ``binary_stats_fused``)."""
        if self.multidim_average != "global" or not ops.use_native(target) or not self._int64_states():
            return False
        sink = self._validation_sink(target) if self.validate_args else None
        if self.validate_args:
            validate(sink, sink is None)
        err_t, err_p = _binary_value_flags(sink, preds)
        states = (self.tp, self.fp, self.tn, self.fn)
        cls_ops.binary_stats_fused(
            preds, target, states, self._scratch(6 * num_labels + cls_ops.GRID_SLOTS, target.device), num_labels, self.threshold,
            self.ignore_index, err_t, err_p,
        )
        return True

    def _update_state(self, tp: Tensor, fp: Tensor, tn: Tensor, fn: Tensor) -> None:
        if self.multidim_average == "samplewise":
            self.tp.append(tp)
            self.fp.append(fp)
            self.tn.append(tn)
            self.fn.append(fn)
        else:
            self.tp += tp
            self.fp += fp
            self.tn += tn
            self.fn += fn

    def _final_state(self) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
        return dim_zero_cat(self.tp), dim_zero_cat(self.fp), dim_zero_cat(self.tn), dim_zero_cat(self.fn)

    def plot(self, val: Optional[Union[Tensor, Sequence[Tensor]]] = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:
        return self._plot(val, ax)


class BinaryStatScores(_AbstractStatScores):
    """tp / fp / tn / fn / support for binary tasks.

    Example:
        >>> import torch
        >>> from torchmetrics_forked_amd.classification import BinaryStatScores
        >>> preds = torch.tensor([0.1, 0.8, 0.6, 0.3, 0.9, 0.2])
        >>> target = torch.tensor([0, 1, 0, 0, 1, 1])
        >>> metric = BinaryStatScores()
        >>> metric(preds, target)
        tensor([2, 1, 2, 1, 3])
    """

    is_differentiable: bool = False
    higher_is_better: Optional[bool] = None
    full_state_update: bool = False

    def __init__(
        self,
        threshold: float = 0.5,
        multidim_average: Literal["global", "samplewise"] = "global",
        ignore_index: Optional[int] = None,
        validate_args: bool = True,
        **kwargs: Any,
    ) -> None:
        super(_AbstractStatScores, self).__init__(**kwargs)
        if validate_args:
            _binary_stat_scores_arg_validation(threshold, multidim_average, ignore_index)
        self.threshold = threshold
        self.multidim_average = multidim_average
        self.ignore_index = ignore_index
        self.validate_args = validate_args
        self._create_state(size=1, multidim_average=multidim_average)

    def _batch_stats(self, preds: Tensor, target: Tensor) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
        if self.validate_args:
            _binary_stat_scores_tensor_validation(
                preds, target, self.multidim_average, self.ignore_index, self._validation_sink(target)
            )
        if self.multidim_average == "global":
            return _binary_stats_fused(preds, target, self.threshold, self.ignore_index)
        preds, target = _binary_stat_scores_format(preds, target, self.threshold, self.ignore_index)
        return _binary_stat_scores_update(preds, target, self.multidim_average)

    def update(self, preds: Tensor, target: Tensor) -> None:
        validate = lambda sink, values: _binary_stat_scores_tensor_validation(  # noqa: E731
            preds, target, self.multidim_average, self.ignore_index, sink, values
        )
        if not self._binary_fused_update(preds, target, 1, validate):
            self._update_state(*self._batch_stats(preds, target))

    def compute(self) -> Tensor:
        tp, fp, tn, fn = self._final_state()
        return _binary_stat_scores_compute(tp, fp, tn, fn, self.multidim_average)


class MulticlassStatScores(_AbstractStatScores):
    """tp / fp / tn / fn / support for multiclass tasks.

    Example:
        >>> import torch
        >>> from torchmetrics_forked_amd.classification import MulticlassStatScores
        >>> metric = MulticlassStatScores(num_classes=3, average=None)
        >>> metric(torch.tensor([2, 1, 0, 1]), torch.tensor([2, 1, 0, 0]))
        tensor([[1, 0, 2, 1, 2],
                [1, 1, 2, 0, 1],
                [1, 0, 3, 0, 1]])
    """

    is_differentiable: bool = False
    higher_is_better: Optional[bool] = None
    full_state_update: bool = False

    def __init__(
        self,
        num_classes: int,
        top_k: int = 1,
        average: Optional[Literal["micro", "macro", "weighted", "none"]] = "macro",
        multidim_average: Literal["global", "samplewise"] = "global",
        ignore_index: Optional[int] = None,
        validate_args: bool = True,
        **kwargs: Any,
    ) -> None:
        super(_AbstractStatScores, self).__init__(**kwargs)
        if validate_args:
            _multiclass_stat_scores_arg_validation(num_classes, top_k, average, multidim_average, ignore_index)
        self.num_classes = num_classes
        self.top_k = top_k
        self.average = average
        self.multidim_average = multidim_average
        self.ignore_index = ignore_index
        self.validate_args = validate_args
        self._create_state(size=1 if (average == "micro" and top_k == 1) else num_classes, multidim_average=multidim_average)

    def _batch_stats(self, preds: Tensor, target: Tensor) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
        if self.validate_args:
            _multiclass_stat_scores_tensor_validation(
                preds, target, self.num_classes, self.multidim_average, self.ignore_index, self._validation_sink(target)
            )
        return _multiclass_stat_scores_update(
            preds, target, self.num_classes, self.top_k, self.average, self.multidim_average, self.ignore_index
        )

    def _fused_update(self, preds: Tensor, target: Tensor) -> bool:
        """GPU fast path for global top-1 stats: validation shape checks on the host, value checks as device flags
        and the counts straight into the states -- one kernel per update instead of a [C, C] temporary plus ~25
        small kernels (csrc/classification.hip ``mc_stat_scores_update``)."""
        if self.multidim_average != "global" or self.top_k != 1 or not self._int64_states():
            return False
        if not ops.use_native(target):
            if not (preds.is_cpu and target.is_cpu and self.tp.is_cpu and ops.load()):  # cls_ops.host_native, inlined
                return False
            # CPU (gloo / plumbing): shape checks here, value check + arg-max + accumulation in one host call
            if self.validate_args:
                _multiclass_stat_scores_tensor_validation(preds, target, self.num_classes, "global", self.ignore_index, None, False)
            p, t = _multiclass_pairs_view(preds, target, self.num_classes)
            cls_ops.mc_stats_host(
                p, t, self.num_classes, (self.tp, self.fp, self.tn, self.fn), self.ignore_index, self.average == "micro",
                self.validate_args,
            )
            return True
        sink = self._validation_sink(target) if self.validate_args else None
        if self.validate_args:
            _multiclass_stat_scores_tensor_validation(
                preds, target, self.num_classes, "global", self.ignore_index, sink, check_values=sink is None
            )
        err_t, err_p = _multiclass_range_flags(sink, preds)
        ticket = self._scratch(cls_ops.GRID_SLOTS, target.device)
        _multiclass_stat_scores_accumulate(
            preds, target, self.num_classes, (self.tp, self.fp, self.tn, self.fn), ticket, self.ignore_index,
            self.average == "micro", err_t, err_p,
        )
        return True

    def update(self, preds: Tensor, target: Tensor) -> None:
        if not self._fused_update(preds, target):
            self._update_state(*self._batch_stats(preds, target))

    def _bootstrap_deltas(self, weights: Tensor, preds: Tensor, target: Tensor) -> Optional[Dict[str, Tensor]]:
        """BootStrapper's weighted path: tp / fp / tn / fn increments of all B resamples at once from the
        resample counts ``weights [B, N]`` -- three weighted scatters over the (target, argmax) pairs instead of B
        resampled updates.  Global top-1 with ``[N, C]`` scores or ``[N]`` labels only (else None: per-copy path)."""
        if self.multidim_average != "global" or self.top_k != 1 or target.ndim != 1 or preds.ndim not in (1, 2):
            return None
        C = self.num_classes
        if self.validate_args:
            _multiclass_stat_scores_tensor_validation(preds, target, C, "global", self.ignore_index)
        p = preds.argmax(1) if preds.ndim == 2 else preds.long()
        t = target.long()
        w = weights.to(t.device, torch.float64)
        keep = (t >= 0) & (t < C) & (p >= 0) & (p < C)
        if self.ignore_index is not None:
            keep &= t != self.ignore_index
        w = w * keep.to(w.dtype)
        tc, pc = t.clamp(0, C - 1), p.clamp(0, C - 1)
        B = w.shape[0]
        cnt_t = torch.zeros(B, C, dtype=w.dtype, device=w.device).index_add_(1, tc, w)
        cnt_p = torch.zeros(B, C, dtype=w.dtype, device=w.device).index_add_(1, pc, w)
        cnt_tp = torch.zeros(B, C, dtype=w.dtype, device=w.device).index_add_(1, tc, w * (tc == pc).to(w.dtype))
        n = w.sum(1, keepdim=True)
        tp, fp, fn = cnt_tp, cnt_p - cnt_tp, cnt_t - cnt_tp
        tn = n - tp - fp - fn
        if self.average == "micro":
            tp, fp, fn, tn = tp.sum(1), fp.sum(1), fn.sum(1), tn.sum(1)
        return {k: v.round().long() for k, v in (("tp", tp), ("fp", fp), ("tn", tn), ("fn", fn))}

    def _fusion_key(self) -> Optional[Tuple]:
        """Collection fusion (ops/fused.py): global top-1 stats derive from the shared argmax pair counts."""
        if self.multidim_average != "global" or self.top_k != 1:
            return None
        return ("multiclass_scores", self.num_classes, self.ignore_index)

    def _fold_states(self) -> Optional[Tuple[Tensor, Tensor, Tensor, Tensor, bool]]:
        """(tp, fp, tn, fn, micro) states the fused plan's ``confmat_fold`` adds into, or None when not fusable."""
        if self.multidim_average != "global" or self.top_k != 1:
            return None
        states = (self.tp, self.fp, self.tn, self.fn)
        if not all(isinstance(s, Tensor) and s.dtype == torch.long and s.is_contiguous() for s in states):
            return None
        return (*states, self.average == "micro")

    def compute(self) -> Tensor:
        tp, fp, tn, fn = self._final_state()
        return _multiclass_stat_scores_compute(tp, fp, tn, fn, self.average, self.multidim_average)


class MultilabelStatScores(_AbstractStatScores):
    """tp / fp / tn / fn / support for multilabel tasks.

    Example:
        >>> import torch
        >>> from torchmetrics_forked_amd.classification import MultilabelStatScores
        >>> preds = torch.tensor([[0.2, 0.9, 0.1], [0.7, 0.4, 0.3], [0.6, 0.8, 0.9]])
        >>> target = torch.tensor([[0, 1, 0], [1, 0, 1], [1, 1, 0]])
        >>> metric = MultilabelStatScores(num_labels=3, average=None)
        >>> metric(preds, target)
        tensor([[2, 0, 1, 0, 2],
                [2, 0, 1, 0, 2],
                [0, 1, 1, 1, 1]])
    """

    is_differentiable: bool = False
    higher_is_better: Optional[bool] = None
    full_state_update: bool = False

    def __init__(
        self,
        num_labels: int,
        threshold: float = 0.5,
        average: Optional[Literal["micro", "macro", "weighted", "none"]] = "macro",
        multidim_average: Literal["global", "samplewise"] = "global",
        ignore_index: Optional[int] = None,
        validate_args: bool = True,
        **kwargs: Any,
    ) -> None:
        super(_AbstractStatScores, self).__init__(**kwargs)
        if validate_args:
            _multilabel_stat_scores_arg_validation(num_labels, threshold, average, multidim_average, ignore_index)
        self.num_labels = num_labels
        self.threshold = threshold
        self.average = average
        self.multidim_average = multidim_average
        self.ignore_index = ignore_index
        self.validate_args = validate_args
        self._create_state(size=num_labels, multidim_average=multidim_average)

    def _batch_stats(self, preds: Tensor, target: Tensor) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
        if self.validate_args:
            _multilabel_stat_scores_tensor_validation(
                preds, target, self.num_labels, self.multidim_average, self.ignore_index, self._validation_sink(target)
            )
        if self.multidim_average == "global":
            return _multilabel_stats_fused(preds, target, self.num_labels, self.threshold, self.ignore_index)
        preds, target = _multilabel_stat_scores_format(preds, target, self.num_labels, self.threshold, self.ignore_index)
        return _multilabel_stat_scores_update(preds, target, self.multidim_average)

    def update(self, preds: Tensor, target: Tensor) -> None:
        validate = lambda sink, values: _multilabel_stat_scores_tensor_validation(  # noqa: E731
            preds, target, self.num_labels, self.multidim_average, self.ignore_index, sink, values
        )
        if not self._binary_fused_update(preds, target, self.num_labels, validate):
            self._update_state(*self._batch_stats(preds, target))

    def compute(self) -> Tensor:
        tp, fp, tn, fn = self._final_state()
        return _multilabel_stat_scores_compute(tp, fp, tn, fn, self.average, self.multidim_average)


def _task_factory(
    task: str,
    binary_cls: Type[Metric],
    multiclass_cls: Type[Metric],
    multilabel_cls: Type[Metric],
    binary_args: tuple,
    multiclass_args: tuple,
    multilabel_args: tuple,
    num_classes: Optional[int],
    num_labels: Optional[int],
    top_k: Optional[int],
    kwargs: dict,
) -> Metric:
    """Shared ``__new__`` body of the task wrappers (reference e.g. ``classification/stat_scores.py:515-546``)."""
    task = ClassificationTask.from_str(task)
    if task == ClassificationTask.BINARY:
        return binary_cls(*binary_args, **kwargs)
    if task == ClassificationTask.MULTICLASS:
        if not isinstance(num_classes, int):
            raise ValueError(f"`num_classes` is expected to be `int` but `{type(num_classes)} was passed.`")
        if top_k is not None and not isinstance(top_k, int):
            raise ValueError(f"`top_k` is expected to be `int` but `{type(top_k)} was passed.`")
        return multiclass_cls(*multiclass_args, **kwargs)
    if task == ClassificationTask.MULTILABEL:
        if not isinstance(num_labels, int):
            raise ValueError(f"`num_labels` is expected to be `int` but `{type(num_labels)} was passed.`")
        return multilabel_cls(*multilabel_args, **kwargs)
    raise ValueError(f"Task {task} not supported!")


class StatScores(_ClassificationTaskWrapper):
    """Task wrapper returning Binary/Multiclass/MultilabelStatScores."""

    def __new__(  # type: ignore[misc]
        cls: Type["StatScores"],
        task: Literal["binary", "multiclass", "multilabel"],
        threshold: float = 0.5,
        num_classes: Optional[int] = None,
        num_labels: Optional[int] = None,
        average: Optional[Literal["micro", "macro", "weighted", "none"]] = "micro",
        multidim_average: Optional[Literal["global", "samplewise"]] = "global",
        top_k: Optional[int] = 1,
        ignore_index: Optional[int] = None,
        validate_args: bool = True,
        **kwargs: Any,
    ) -> Metric:
        assert multidim_average is not None  # noqa: S101
        kwargs.update({"multidim_average": multidim_average, "ignore_index": ignore_index, "validate_args": validate_args})
        return _task_factory(
            task, BinaryStatScores, MulticlassStatScores, MultilabelStatScores,
            (threshold,), (num_classes, top_k, average), (num_labels, threshold, average),
            num_classes, num_labels, top_k, kwargs,
        )
