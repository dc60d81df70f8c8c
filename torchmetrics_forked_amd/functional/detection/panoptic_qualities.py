"""Panoptic Quality and Modified Panoptic Quality (API parity: reference
``functional/detection/panoptic_qualities.py:29-160``); batched segment statistics in
``_panoptic_quality_common``."""
from typing import Collection

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


def _pq(preds: Tensor, target: Tensor, things: Collection[int], stuffs: Collection[int], allow_unknown: bool, modified: bool) -> Tensor:
    things, stuffs = _parse_categories(things, stuffs)
    _validate_inputs(preds, target)
    void_color = _get_void_color(things, stuffs)
    cat_map = _get_category_id_to_continuous_id(things, stuffs)
    fp = _prepocess_inputs(things, stuffs, preds, void_color, allow_unknown)
    ft = _prepocess_inputs(things, stuffs, target, void_color, True)
    stats = _panoptic_quality_update(fp, ft, cat_map, void_color, modified_metric_stuffs=stuffs if modified else None)
    return _panoptic_quality_compute(*stats)


def panoptic_quality(
    preds: Tensor,
    target: Tensor,
    things: Collection[int],
    stuffs: Collection[int],
    allow_unknown_preds_category: bool = False,
) -> Tensor:
    """PQ over ``[B, *spatial, 2]`` ``(category_id, instance_id)`` maps."""
    return _pq(preds, target, things, stuffs, allow_unknown_preds_category, modified=False)


def modified_panoptic_quality(
    preds: Tensor,
    target: Tensor,
    things: Collection[int],
    stuffs: Collection[int],
    allow_unknown_preds_category: bool = False,
) -> Tensor:
    """PQ with the modified (segment-free) formula for stuff categories (Porzi et al.)."""
    return _pq(preds, target, things, stuffs, allow_unknown_preds_category, modified=True)
