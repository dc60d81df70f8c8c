"""Fused update plans for ``MetricCollection`` ("metrics reading the same inputs share one
fused kernel").

A plan groups collection members whose ``_fusion_key()`` matches and for which a fused kernel exists.  The
plan is attempted on every update; if the inputs do not qualify (e.g. fp32 scores, thresholds set) it returns
``False`` and the collection falls back to per-metric updates, so results never depend on fusion.

Implemented plan:
  * ``multiclass_scores``: one curve metric on the exact-histogram path (``MulticlassAUROC`` /
    ``MulticlassAveragePrecision`` / ``MulticlassROC`` / ``MulticlassPrecisionRecallCurve``) + any number of
    ``MulticlassConfusionMatrix`` members -> one pass over the ``[N, C]`` scores computes the softmax code
    histogram *and* the argmax confusion matrix (``tmx::curve_hist_update`` with ``confmat``).
"""
from typing import Any, Dict, List, Tuple

import torch
from torch import Tensor

from torchmetrics_forked_amd.functional.classification import _curve_engine as eng


class _MulticlassScoresPlan:
    def __init__(self, names: List[str], curve_name: str, confmat_names: List[str]) -> None:
        self.names = names
        self.curve_name = curve_name
        self.confmat_names = confmat_names

    def run(self, members: Dict[str, Any], args: Tuple, kwargs: Dict[str, Any]) -> bool:
        if self.curve_name not in members or len(members) < 2:
            return False
        preds = kwargs.get("preds", args[0] if len(args) > 0 else None)
        target = kwargs.get("target", args[1] if len(args) > 1 else None)
        if not isinstance(preds, Tensor) or not isinstance(target, Tensor):
            return False
        curve = members[self.curve_name]
        if preds.dtype not in eng.HIST_DTYPES or preds.ndim != 2 or not curve._hist_ok(preds):
            return False
        confmats = [members[n] for n in self.confmat_names if n in members]
        # validation: host-side shape checks per member; the target range check runs inside the fused kernel
        # (device flag shared by every member's deferred sink, raised at compute) or eagerly on CPU.
        from torchmetrics_forked_amd.functional.classification.precision_recall_curve import TARGET_RANGE_MSG

        err = curve._validate_fused(preds, target)
        for cm in confmats:
            cm._validate(preds, target, check_values=err is None)
            if err is not None and cm.validate_args:
                cm._validation_sink(target).attach(RuntimeError, TARGET_RANGE_MSG, err)
        if len(confmats) == 1:
            delta = confmats[0].confmat  # accumulate straight into the state
        else:
            delta = torch.zeros_like(confmats[0].confmat)
        for m in [curve, *confmats]:
            m._computed = None
            m._update_count += 1
        curve._curve_update(preds, target, confmat_out=delta, err_flag=err)
        side = curve.__dict__.get("_side_event")
        if side is not None:  # the side-stream class pass also adds rare rows into the confusion matrix
            if len(confmats) > 1:
                curve._join_side_work()
            else:
                confmats[0].__dict__["_side_event"] = side
        if len(confmats) > 1:
            for cm in confmats:
                cm.confmat += delta
        return True


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
        if key[0] != "multiclass_scores" or len(names) < 2:
            continue
        curves = [n for n in names if hasattr(modules[n], "_curve_update")]
        confmats = [n for n in names if n not in curves and hasattr(modules[n], "confmat")]
        if len(curves) >= 1 and confmats:
            plans.append(_MulticlassScoresPlan([curves[0], *confmats], curves[0], confmats))
    return plans
