"""PanopticQuality / ModifiedPanopticQuality modules (API parity: reference ``detection/panoptic_qualities.py``).

States are the reference's four per-category ``sum`` vectors (fp64 IoU sum, int32 TP/FP/FN), so they sync with
one coalesced all-reduce."""
from typing import Any, Collection, Optional, Sequence, Union

import torch
from torch import Tensor

from torchmetrics_forked_amd.functional.detection._panoptic_quality_common import (
    _get_category_id_to_continuous_id,
    _get_void_color,
    _panoptic_quality_compute,
    _panoptic_quality_update,
    _parse_categories,
    _prepocess_inputs,
    _validate_inputs,
)
from torchmetrics_forked_amd.metric import Metric
from torchmetrics_forked_amd.utilities.plot import _AX_TYPE, _PLOT_OUT_TYPE


class PanopticQuality(Metric):
    """Panoptic Quality over ``[B, *spatial, 2]`` ``(category_id, instance_id)`` maps."""

    is_differentiable: bool = False
    higher_is_better: bool = True
    full_state_update: bool = False
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0
    _modified: bool = False

    iou_sum: Tensor
    true_positives: Tensor
    false_positives: Tensor
    false_negatives: Tensor

    def __init__(
        self,
        things: Collection[int],
        stuffs: Collection[int],
        allow_unknown_preds_category: bool = False,
        **kwargs: Any,
    ) -> None:
        super().__init__(**kwargs)
        things, stuffs = _parse_categories(things, stuffs)
        self.things = things
        self.stuffs = stuffs
        self.void_color = _get_void_color(things, stuffs)
        self.cat_id_to_continuous_id = _get_category_id_to_continuous_id(things, stuffs)
        self.allow_unknown_preds_category = allow_unknown_preds_category
        k = len(things) + len(stuffs)
        self.add_state("iou_sum", default=torch.zeros(k, dtype=torch.double), dist_reduce_fx="sum")
        self.add_state("true_positives", default=torch.zeros(k, dtype=torch.int), dist_reduce_fx="sum")
        self.add_state("false_positives", default=torch.zeros(k, dtype=torch.int), dist_reduce_fx="sum")
        self.add_state("false_negatives", default=torch.zeros(k, dtype=torch.int), dist_reduce_fx="sum")

    def update(self, preds: Tensor, target: Tensor) -> None:
        _validate_inputs(preds, target)
        fp = _prepocess_inputs(self.things, self.stuffs, preds, self.void_color, self.allow_unknown_preds_category)
        ft = _prepocess_inputs(self.things, self.stuffs, target, self.void_color, True)
        iou_sum, tp, fp_, fn = _panoptic_quality_update(
            fp, ft, self.cat_id_to_continuous_id, self.void_color,
            modified_metric_stuffs=self.stuffs if self._modified else None,
        )
        self.iou_sum += iou_sum
        self.true_positives += tp
        self.false_positives += fp_
        self.false_negatives += fn

    def compute(self) -> Tensor:
        return _panoptic_quality_compute(self.iou_sum, self.true_positives, self.false_positives, self.false_negatives)

    def plot(
        self, val: Optional[Union[Tensor, Sequence[Tensor]]] = None, ax: Optional[_AX_TYPE] = None
    ) -> _PLOT_OUT_TYPE:
        return self._plot(val, ax)


class ModifiedPanopticQuality(PanopticQuality):
    """Modified Panoptic Quality: stuff categories scored by IoU sum over target segments (no matching)."""

    _modified: bool = True
