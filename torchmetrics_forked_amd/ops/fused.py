"""Fused update plans for ``MetricCollection`` ("metrics reading the same inputs share one
fused kernel"; the reference's compute groups, ``collections.py:200-307``, only share the states of metrics that
would compute identical states).

A plan groups collection members whose ``_fusion_key()`` matches.  It is attempted on every update (and on
``forward``); if the inputs do not qualify it returns ``False`` and the collection falls back to per-metric updates,
so results never depend on fusion.

``multiclass_scores`` plan (key ``("multiclass_scores", C, ignore_index)``) over
  * at most one curve metric on the exact-histogram path (``MulticlassAUROC`` / ``AveragePrecision`` / ``ROC`` /
    ``PrecisionRecallCurve``, bf16 / fp16 scores),
  * any number of confusion-matrix members (``MulticlassConfusionMatrix``),
  * any number of StatScores-family members (``MulticlassAccuracy`` / ``Precision`` / ``Recall`` / ``F1Score`` /
    ``FBetaScore`` / ``Specificity`` / ``HammingDistance`` / ``StatScores``; global, top-1).
One pass over the ``[N, C]`` scores -- the curve's row pass (softmax code histogram + argmax pairs) or, without a
curve member, the argmax pair stream -- counts the batch's (target, argmax) pairs into a scratch ``[C, C]`` matrix;
``tmx::confmat_fold`` (csrc/fused.hip) then adds it to every confusion-matrix state and turns its diagonal / row /
column sums into every stat member's tp / fp / tn / fn.  With a single confusion-matrix member and no stat member
the pass accumulates straight into that member's state.

``image_pair`` plan (key ``("image_pair",)``) over one ``StructuralSimilarityIndexMeasure`` (fixed ``data_range``,
scalar reduction) and any number of ``PeakSignalNoiseRatio`` members (fixed ``data_range``, ``dim=None``): the SSIM
kernel (csrc/image.hip ``ssim_v2_kernel<KS, true>``) adds every input pixel's squared error while it stages the two
images, so PSNR costs no second pass over them (256 x 3 x 1024^2 fp32: 6.4 GB not re-read).
"""
from typing import Any, Dict, List, Optional, Tuple

import torch
from torch import Tensor

from torchmetrics_forked_amd import ops
from torchmetrics_forked_amd.functional.classification import _curve_engine as eng


_NAMES: Optional[Tuple[Any, ...]] = None


def _validation_names() -> Tuple[Any, ...]:
    """The validation helpers ``run`` needs, imported once (a function-level import costs ~1 us per update)."""
    global _NAMES
    if _NAMES is None:
        from torchmetrics_forked_amd.functional.classification.precision_recall_curve import TARGET_RANGE_MSG
        from torchmetrics_forked_amd.functional.classification.stat_scores import (
            _TARGET_RANGE_MSG,
            _multiclass_range_flags,
            _multiclass_stat_scores_tensor_validation,
        )

        _NAMES = (TARGET_RANGE_MSG, _TARGET_RANGE_MSG, _multiclass_range_flags, _multiclass_stat_scores_tensor_validation)
    return _NAMES


def _stat_fusable(m: Any) -> bool:
    return hasattr(m, "_fold_states") and m._fold_states() is not None


class _MulticlassScoresPlan:
    def __init__(self, curve_name: Optional[str], confmat_names: List[str], stat_names: List[str]) -> None:
        self.curve_name = curve_name
        self.confmat_names = confmat_names
        self.stat_names = stat_names
        self.names = ([curve_name] if curve_name else []) + confmat_names + stat_names
        self._scratch: Dict[torch.device, Tuple[Tensor, Tensor]] = {}

    def _buffers(self, C: int, device: torch.device) -> Tuple[Tensor, Tensor]:
        buf = self._scratch.get(device)
        if buf is None or buf[0].shape[0] != C:
            # zeroed once; confmat_fold leaves both zero again after every batch
            buf = (torch.zeros(C, C, dtype=torch.long, device=device), torch.zeros(3 * C + 1, dtype=torch.long, device=device))  # class sums + workgroup ticket
            self._scratch[device] = buf
        return buf

    def run(self, members: Dict[str, Any], args: Tuple, kwargs: Dict[str, Any]) -> List[str]:
        """Update the qualifying members with one pass; returns their names (empty: nothing was done)."""
        if len(members) < 2:
            return []
        preds = kwargs.get("preds", args[0] if len(args) > 0 else None)
        target = kwargs.get("target", args[1] if len(args) > 1 else None)
        if not isinstance(preds, Tensor) or not isinstance(target, Tensor) or not preds.is_floating_point():
            return []
        if preds.ndim != 2 or target.ndim != 1 or target.device != preds.device or not ops.use_native(preds):
            return []
        curve = members.get(self.curve_name) if self.curve_name else None
        if curve is not None and (preds.dtype not in eng.HIST_DTYPES or not curve._hist_ok(preds)):
            curve = None
        confmats = [members[n] for n in self.confmat_names if n in members]
        stats = [members[n] for n in self.stat_names if n in members and _stat_fusable(members[n])]
        if len(confmats) + len(stats) + (curve is not None) < 2 or len(confmats) > 8 or len(stats) > 8:
            return []
        C = preds.shape[1]
        dev = preds.device
        for cm in confmats:
            if cm.num_classes != C or cm.confmat.dtype != torch.long or cm.confmat.device != dev:
                return []  # states on another device: the members' own updates raise the device error
        for st in stats:
            if st.num_classes != C:
                return []
            for k in ("tp", "fp", "tn", "fn"):
                v = getattr(st, k, None)
                if isinstance(v, Tensor) and v.numel() > 0 and v.device != dev:
                    return []
        TARGET_RANGE_MSG, _TARGET_RANGE_MSG, _multiclass_range_flags, _multiclass_stat_scores_tensor_validation = _validation_names()

        # validation: host-side shape checks per member; the target range check runs inside the fused pass (one
        # device flag shared by every member's deferred sink, raised at compute) or eagerly on CPU
        if curve is not None:
            err = curve._validate_fused(preds, target)
        else:
            lead = (confmats + stats)[0]
            err = _multiclass_range_flags(lead._validation_sink(target), preds)[0] if lead.validate_args else None
        for cm in confmats:
            cm._validate(preds, target, check_values=err is None)
        for st in stats:
            if st.validate_args:
                _multiclass_stat_scores_tensor_validation(
                    preds, target, st.num_classes, "global", st.ignore_index, st._validation_sink(target), check_values=err is None
                )
        pending: List[Tuple[Tensor, Tensor]] = []
        if err is not None:
            for group, msg in ((confmats, TARGET_RANGE_MSG), (stats, _TARGET_RANGE_MSG)):
                for m in group:
                    if not m.validate_args:
                        continue
                    sink = m._deferred if m._deferred is not None else m._validation_sink(target)
                    prev = sink._flags.get((RuntimeError, msg))
                    if prev is err:
                        continue  # attached by an earlier batch (the steady state)
                    if prev is None:
                        sink.attach(RuntimeError, msg, err)
                    else:
                        pending.append((prev, err))

        direct = len(confmats) == 1 and not stats
        if direct:
            delta, sums = confmats[0].confmat, None
        else:
            delta, sums = self._buffers(C, preds.device)
        updated = ([curve] if curve is not None else []) + confmats + stats
        for m in updated:
            d = m.__dict__  # plain attributes: no nn.Module __setattr__ per member per update
            d["_computed"] = None
            d["_update_count"] += 1
        if curve is not None:
            # update lanes (side streams) only when no fold runs after the pass on the caller's stream
            curve._curve_update(preds, target, confmat_out=delta, err_flag=err, lanes_ok=direct)
            join = curve.__dict__.get("_side_event")
            if join is not None:  # the confusion-matrix state is written on the curve's lanes: its consumers join them
                for cm in confmats:
                    if cm.__dict__.get("_side_event") is None:
                        cm.__dict__["_side_event"] = join
        else:
            from torchmetrics_forked_amd.ops import classification as cls_ops

            ii = (confmats + stats)[0].ignore_index
            cls_ops.mc_confmat_update(preds, target, delta, ii, err, None)
        if not direct:
            states: List[Tensor] = []
            micro: List[int] = []
            for st in stats:
                tp, fp, tn, fn, is_micro = st._fold_states()
                states += [tp, fp, tn, fn]
                micro.append(int(is_micro))
            torch.ops.tmx.confmat_fold(delta, [cm.confmat for cm in confmats], states, micro, sums)
        # a member whose sink already held a range flag of its own gets the shared flag OR-ed in after the pass
        for prev, e in pending:
            prev.bitwise_or_(e)
        ids = {id(u) for u in updated}
        return [n for n, m in members.items() if id(m) in ids]


class _ImagePairPlan:
    def __init__(self, ssim_name: str, psnr_names: List[str]) -> None:
        self.ssim_name = ssim_name
        self.psnr_names = psnr_names
        self.names = [ssim_name] + psnr_names

    def run(self, members: Dict[str, Any], args: Tuple, kwargs: Dict[str, Any]) -> List[str]:
        ssim = members.get(self.ssim_name)
        psnrs = [members[n] for n in self.psnr_names if n in members]
        if ssim is None or not psnrs:
            return []
        preds = kwargs.get("preds", args[0] if len(args) > 0 else None)
        target = kwargs.get("target", args[1] if len(args) > 1 else None)
        if not isinstance(preds, Tensor) or not isinstance(target, Tensor) or preds.ndim != 4 or preds.dtype != torch.float32:
            return []
        if preds.shape != target.shape or not ops.use_native(preds) or torch.is_grad_enabled() and preds.requires_grad:
            return []
        if any(p.sum_squared_error.device != preds.device for p in psnrs):
            return []
        sse: List[Tensor] = []
        for m in [ssim] + psnrs:
            m._computed = None
            m._update_count += 1
        ssim._fused_update(preds, target, sse)
        for p in psnrs:
            if sse:
                p._fused_add(sse[0], preds.numel())
            else:  # the kernel could not take the inputs (window / shape): PSNR's own pass
                p._update_count -= 1
                p.update(preds, target)
        return [n for n, m in members.items() if m is ssim or any(m is p for p in psnrs)]


def build_fused_plans(modules: Dict[str, Any]) -> List[Any]:
    groups: Dict[Tuple, List[str]] = {}
    for name, m in modules.items():
        key_fn = getattr(m, "_fusion_key", None)
        if key_fn is None:
            continue
        key = key_fn()
        if key is not None:
            groups.setdefault(key, []).append(name)
    plans: List[Any] = []
    for key, names in groups.items():
        if key[0] == "image_pair":
            ssims = [n for n in names if hasattr(modules[n], "_fused_update")]
            psnrs = [n for n in names if hasattr(modules[n], "_fused_add")]
            if ssims and psnrs:
                plans.append(_ImagePairPlan(ssims[0], psnrs))
            continue
        if key[0] != "multiclass_scores" or len(names) < 2:
            continue
        curves = [n for n in names if hasattr(modules[n], "_curve_update")]
        stats = [n for n in names if n not in curves and hasattr(modules[n], "_fold_states")]
        confmats = [n for n in names if n not in curves and n not in stats and hasattr(modules[n], "confmat")]
        if len(curves[:1]) + len(confmats) + len(stats) >= 2 and (confmats or stats):
            plans.append(_MulticlassScoresPlan(curves[0] if curves else None, confmats, stats))
    return plans
