"""Detection input helpers (API parity: reference ``detection/helpers.py:19-103``)."""
from typing import Dict, Literal, Sequence, Tuple, Union

from torch import Tensor

_NAME_MAP = {"bbox": "boxes", "segm": "masks"}


def _input_validator(
    preds: Sequence[Dict[str, Tensor]],
    targets: Sequence[Dict[str, Tensor]],
    iou_type: Union[Literal["bbox", "segm"], Tuple[Literal["bbox", "segm"]]] = "bbox",
    ignore_score: bool = False,
) -> None:
    """Check the list-of-dicts detection input format (same error messages as the reference)."""
    if isinstance(iou_type, str):
        iou_type = (iou_type,)
    if any(tp not in _NAME_MAP for tp in iou_type):
        raise Exception(f"IOU type {iou_type} is not supported")
    keys = [_NAME_MAP[tp] for tp in iou_type]
    if not isinstance(preds, Sequence):
        raise ValueError(f"Expected argument `preds` to be of type Sequence, but got {preds}")
    if not isinstance(targets, Sequence):
        raise ValueError(f"Expected argument `target` to be of type Sequence, but got {targets}")
    if len(preds) != len(targets):
        raise ValueError(
            f"Expected argument `preds` and `target` to have the same length, but got {len(preds)} and {len(targets)}"
        )
    for k in [*keys, "labels"] + ([] if ignore_score else ["scores"]):
        if any(k not in p for p in preds):
            raise ValueError(f"Expected all dicts in `preds` to contain the `{k}` key")
    for k in [*keys, "labels"]:
        if any(k not in t for t in targets):
            raise ValueError(f"Expected all dicts in `target` to contain the `{k}` key")
    for k in keys:
        if not all(isinstance(p[k], Tensor) for p in preds):
            raise ValueError(f"Expected all {k} in `preds` to be of type Tensor")
    if not ignore_score and not all(isinstance(p["scores"], Tensor) for p in preds):
        raise ValueError("Expected all scores in `preds` to be of type Tensor")
    if not all(isinstance(p["labels"], Tensor) for p in preds):
        raise ValueError("Expected all labels in `preds` to be of type Tensor")
    for k in keys:
        if not all(isinstance(t[k], Tensor) for t in targets):
            raise ValueError(f"Expected all {k} in `target` to be of type Tensor")
    if not all(isinstance(t["labels"], Tensor) for t in targets):
        raise ValueError("Expected all labels in `target` to be of type Tensor")
    for i, item in enumerate(targets):
        for k in keys:
            if item[k].size(0) != item["labels"].size(0):
                raise ValueError(
                    f"Input '{k}' and labels of sample {i} in targets have a"
                    f" different length (expected {item[k].size(0)} labels, got {item['labels'].size(0)})"
                )
    if ignore_score:
        return
    for i, item in enumerate(preds):
        for k in keys:
            if not (item[k].size(0) == item["labels"].size(0) == item["scores"].size(0)):
                raise ValueError(
                    f"Input '{k}', labels and scores of sample {i} in predictions have a"
                    f" different length (expected {item[k].size(0)} labels and scores,"
                    f" got {item['labels'].size(0)} labels and {item['scores'].size(0)})"
                )


def _fix_empty_tensors(boxes: Tensor) -> Tensor:
    """Give empty 1-d box tensors a leading dim so they concatenate/sync like ``[0, 4]`` tensors."""
    if boxes.numel() == 0 and boxes.ndim == 1:
        return boxes.unsqueeze(0)
    return boxes


def _validate_iou_type_arg(iou_type: Union[Literal["bbox", "segm"], Tuple[str]] = "bbox") -> Tuple[str]:
    allowed = ("segm", "bbox")
    if isinstance(iou_type, str):
        iou_type = (iou_type,)
    if any(tp not in allowed for tp in iou_type):
        raise ValueError(f"Expected argument `iou_type` to be one of {allowed} or a list of, but got {iou_type}")
    return tuple(iou_type)
