"""Mean average precision / recall for object detection (API parity: reference ``detection/mean_ap.py:76-1033``).

Same constructor, states (nine ``None``-reduced per-image lists), output keys and COCO semantics as the
reference, but no COCO JSON round trip and no pycocotools: ``compute`` flattens the per-image lists into one
row per box and hands them to the native evaluator ``tmx::coco_evaluate`` (C++ evaluateImg + accumulate,
parallel over categories; csrc/coco_eval.cpp).  Segmentation IoUs are computed on the metric's device with the
IoU kernel and passed in as per-image matrices.  Masks are stored as the reference stores them — per image a tuple
of ``((H, W), counts)`` COCO RLE entries (``mean_ap.py:811-816``) — but encoded by the GPU kernels of
``csrc/rle.hip`` (one launch group per update batch; only the strings reach the host), and segm IoUs of all images
come from one decode + one tiled popcount launch per mask size (``_mask_utils.rle_segm_ious``).

``backend`` only selects the summary convention: ``"pycocotools"`` evaluates ``map`` (stats[0]) at
``maxDets == 100`` (``-1`` when 100 is not among ``max_detection_thresholds``, as the official tool does),
``"faster_coco_eval"`` at the largest threshold.

Documented deviation: ``average="micro"`` evaluates a single category 0 (the reference keeps the original
category ids in the COCO dataset while relabelling every annotation to 0, which yields ``-1`` everywhere when 0
is not one of the labels).
"""
import itertools
import json
import os
import operator
from typing import ClassVar, Any, Dict, List, Literal, Optional, Sequence, Tuple, Union

import numpy as np
import torch
from torch import Tensor

from torchmetrics_forked_amd import ops
from torchmetrics_forked_amd.detection._mask_utils import (
    encode_mask_batch,
    rle_segm_ious,
    rle_state_area,
    segmentation_to_mask,
)
from torchmetrics_forked_amd.detection.helpers import _fix_empty_tensors, _input_validator, _validate_iou_type_arg
from torchmetrics_forked_amd.functional.detection._box_ops import box_convert
from torchmetrics_forked_amd.metric import Metric
from torchmetrics_forked_amd.utilities import rank_zero_warn
from torchmetrics_forked_amd.utilities.arena import StateArena
from torchmetrics_forked_amd.utilities.plot import _AX_TYPE, _PLOT_OUT_TYPE

_AREA_RANGES = ((0.0, 1e5**2), (0.0, 32.0**2), (32.0**2, 96.0**2), (96.0**2, 1e5**2))
_STAT_NAMES = (
    "map", "map_50", "map_75", "map_small", "map_medium", "map_large",
    "mar_1", "mar_10", "mar_100", "mar_small", "mar_medium", "mar_large",
)


class _EvalResult:
    __slots__ = ("precision", "recall", "iou_values", "iou_index", "cat_ids", "num_images", "overflow")

    def __init__(self, precision: Tensor, recall: Tensor, iou_values: Tensor, iou_index: Tensor, cat_ids: List[int],
                 num_images: int, overflow: Optional[Tensor] = None):
        self.precision, self.recall, self.iou_values, self.iou_index, self.cat_ids, self.num_images = (
            precision, recall, iou_values, iou_index, cat_ids, num_images,
        )
        # device flag of the GPU evaluator: a (image, class) pair past its ground-truth limit (the tables are then
        # invalid and the host evaluator reruns; read together with the summary tables, no extra synchronisation)
        self.overflow = overflow


def _h2d_many(lists: Sequence[Sequence[int]], like: Tensor) -> List[Tensor]:
    """Several host int lists as int64 tensors on ``like``'s device in ONE asynchronous copy through a reused pinned
    buffer (``tmx::upload_i64``): a ``torch.tensor(..., device=cuda)`` copy from pageable memory waits for every
    kernel queued before it, and fresh pinned memory per call costs more than the copy."""
    # (np.fromiter over a chain: 2.6x a list comprehension + torch.tensor for 6K ints)
    flat = torch.from_numpy(np.fromiter(itertools.chain.from_iterable(lists), dtype=np.int64, count=sum(map(len, lists))))
    if like.is_cuda and ops.load():
        flat = torch.ops.tmx.upload_i64(flat, like)
    else:
        flat = flat.to(like.device)
    return list(flat.split([len(lst) for lst in lists]))


class MeanAveragePrecision(Metric):
    """COCO mAP / mAR for boxes (``iou_type="bbox"``) and/or instance masks (``"segm"``)."""

    is_differentiable: bool = False
    higher_is_better: Optional[bool] = True
    full_state_update: bool = True
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0

    # TorchScript-facing declarations (as the reference's ``mean_ap.py:325-350``): the mask states actually hold one
    # tuple of ``((H, W), rle bytes)`` per image, which the JIT type system cannot express; ``update`` / ``compute`` are
    # ``torch.jit.unused`` in script, so only the attribute types must be inferable
    detection_box: List[Tensor]
    detection_mask: List[Tensor]
    detection_scores: List[Tensor]
    detection_labels: List[Tensor]
    groundtruth_box: List[Tensor]
    groundtruth_mask: List[Tensor]
    groundtruth_labels: List[Tensor]
    groundtruth_crowds: List[Tensor]
    groundtruth_area: List[Tensor]

    warn_on_many_detections: bool = True

    # host-side evaluation caches (segm IoU blocks, class-sharded flat states): not module state, invisible to script
    __jit_ignored_attributes__: ClassVar[List[str]] = ["device", "_fast_update", "_segm_cache", "_shard_flat", "_flat_cache", "_param_cache"]

    def __init__(
        self,
        box_format: Literal["xyxy", "xywh", "cxcywh"] = "xyxy",
        iou_type: Union[Literal["bbox", "segm"], Tuple[str]] = "bbox",
        iou_thresholds: Optional[List[float]] = None,
        rec_thresholds: Optional[List[float]] = None,
        max_detection_thresholds: Optional[List[int]] = None,
        class_metrics: bool = False,
        extended_summary: bool = False,
        average: Literal["macro", "micro"] = "macro",
        backend: Literal["pycocotools", "faster_coco_eval"] = "pycocotools",
        **kwargs: Any,
    ) -> None:
        super().__init__(**kwargs)
        allowed = ("xyxy", "xywh", "cxcywh")
        if box_format not in allowed:
            raise ValueError(f"Expected argument `box_format` to be one of {allowed} but got {box_format}")
        self.box_format = box_format
        self.iou_type = _validate_iou_type_arg(iou_type)
        if iou_thresholds is not None and not isinstance(iou_thresholds, list):
            raise ValueError(
                f"Expected argument `iou_thresholds` to either be `None` or a list of floats but got {iou_thresholds}"
            )
        self.iou_thresholds = iou_thresholds or torch.linspace(0.5, 0.95, round((0.95 - 0.5) / 0.05) + 1).tolist()
        if rec_thresholds is not None and not isinstance(rec_thresholds, list):
            raise ValueError(
                f"Expected argument `rec_thresholds` to either be `None` or a list of floats but got {rec_thresholds}"
            )
        self.rec_thresholds = rec_thresholds or torch.linspace(0.0, 1.00, round(1.00 / 0.01) + 1).tolist()
        if max_detection_thresholds is not None and not isinstance(max_detection_thresholds, list):
            raise ValueError(
                f"Expected argument `max_detection_thresholds` to either be `None` or a list of ints"
                f" but got {max_detection_thresholds}"
            )
        max_det, _ = torch.sort(torch.tensor(max_detection_thresholds or [1, 10, 100], dtype=torch.int))
        self.max_detection_thresholds = max_det.tolist()
        if not isinstance(class_metrics, bool):
            raise ValueError("Expected argument `class_metrics` to be a boolean")
        self.class_metrics = class_metrics
        if not isinstance(extended_summary, bool):
            raise ValueError("Expected argument `extended_summary` to be a boolean")
        self.extended_summary = extended_summary
        if average not in ("macro", "micro"):
            raise ValueError(f"Expected argument `average` to be one of ('macro', 'micro') but got {average}")
        self.average = average
        if backend not in ("pycocotools", "faster_coco_eval"):
            raise ValueError(
                f"Expected argument `backend` to be one of ('pycocotools', 'faster_coco_eval') but got {backend}"
            )
        self.backend = backend

        for name in (
            "detection_box", "detection_mask", "detection_scores", "detection_labels", "groundtruth_box",
            "groundtruth_mask", "groundtruth_labels", "groundtruth_crowds", "groundtruth_area",
        ):
            self.add_state(name, default=[], dist_reduce_fx=None)

    # ------------------------------------------------------------------------------------------------------
    # update
    # ------------------------------------------------------------------------------------------------------
    def update(self, preds: List[Dict[str, Tensor]], target: List[Dict[str, Tensor]]) -> None:
        """Append one batch of images.  Box conversion runs once over the whole batch (one ``cat`` + one convert,
        then per-image views), and missing ``iscrowd`` / ``area`` entries share one zero buffer, so the per-image
        cost is list bookkeeping only (the reference converts and allocates per image, ``mean_ap.py:501-540``)."""
        if self._update_batched(preds, target):
            return
        _input_validator(preds, target, iou_type=self.iou_type)
        limit = self.max_detection_thresholds[-1]
        if "bbox" in self.iou_type:
            det_boxes = self._convert_boxes([item["boxes"] for item in preds])
            if self.warn_on_many_detections and any(len(b) > limit for b in det_boxes):
                _warning_on_too_many_detections(limit)
            self.detection_box.extend(det_boxes)
            self.groundtruth_box.extend(self._convert_boxes([item["boxes"] for item in target]))
        if "segm" in self.iou_type:
            det_masks = encode_mask_batch([item["masks"] for item in preds])
            if self.warn_on_many_detections and "bbox" not in self.iou_type and any(len(m) > limit for m in det_masks):
                _warning_on_too_many_detections(limit)
            self.detection_mask.extend(det_masks)
            self.groundtruth_mask.extend(encode_mask_batch([item["masks"] for item in target]))
        self.detection_labels.extend(item["labels"] for item in preds)
        self.detection_scores.extend(item["scores"] for item in preds)
        labels = [item["labels"] for item in target]
        self.groundtruth_labels.extend(labels)
        self.groundtruth_crowds.extend(self._optional_column(target, "iscrowd", labels))
        self.groundtruth_area.extend(self._optional_column(target, "area", labels))

    def _update_batched(self, preds: Any, target: Any) -> bool:
        """Box-only batches of regular images (every image's boxes ``[k, 4]`` and 1-d labels / scores of ``k`` rows, one
        device, ``iscrowd`` / ``area`` given for all images or for none) in O(1) launches and no per-image tensor
        calls: each column is concatenated once, checked once (per-image row counts compared as Python lists), and
        appended with ``StateArena.extend_rows`` as one run, its per-image items being views of that run.  Anything
        else -- a missing key, a non-tensor, a length mismatch, an empty image, segm -- returns False, and the
        per-image path validates it with the reference's messages (``detection/helpers.py``)."""
        if self.iou_type != ("bbox",) or type(preds) is not list or type(target) is not list or len(preds) != len(target) or not preds:
            return False
        states = (self.detection_box, self.detection_scores, self.detection_labels, self.groundtruth_box,
                  self.groundtruth_labels, self.groundtruth_crowds, self.groundtruth_area)
        if not all(isinstance(st, StateArena) for st in states):
            return False
        try:
            pym = ops.py_module()
            if pym is not None:
                # one C pass per list straight over the dicts (csrc/py_columns.cpp): per column one dtype / device /
                # shape, equal row counts across an item's columns, and the concatenation (a view when the items are
                # consecutive rows of one batch tensor); a torch.ops call would box every tensor of each column list
                rp = pym.cat_dict_columns(preds, _PRED_KEYS, _PRED_WIDTHS)
                rt = pym.cat_dict_columns(target, _GT_KEYS, _GT_WIDTHS) if rp is not None else None
                if rt is None:
                    return False
                (flats, dn), (gcols, gn) = rp, rt
                flats = [*flats, gcols[0], gcols[1]]
                crowd, area = gcols[2], gcols[3]
            else:
                # C-level column extraction (map + itemgetter: ~2x a comprehension per 512-image batch)
                cols = (list(map(_BOXES, preds)), list(map(_SCORES, preds)), list(map(_LABELS, preds)),
                        list(map(_BOXES, target)), list(map(_LABELS, target)))
                extra = (_optional_col(target, "iscrowd"), _optional_col(target, "area"))
                n_crowd, n_area = extra[0] is not None, extra[1] is not None
                db, ds, dl, gb, gl = cols
                dn = [t.shape[0] for t in dl]  # (Tensor.__len__ is a Python-level method: 5x the cost of .shape)
                gn = [t.shape[0] for t in gl]
                if dn != [t.shape[0] for t in db] or dn != [t.shape[0] for t in ds] or gn != [t.shape[0] for t in gb] or 0 in dn or 0 in gn:
                    return False
                # one dtype per column: a concatenation would promote mixed images, where the per-image path (and the
                # reference) keeps each image's own tensors
                if any(len({t.dtype for t in col}) != 1 for col in cols):
                    return False
                flats = [torch.cat(col) for col in cols]
                crowd = torch.cat(extra[0]) if n_crowd else None
                area = torch.cat(extra[1]) if n_area else None
        except (KeyError, TypeError, RuntimeError, ValueError, IndexError, AttributeError):
            return False
        det_box, det_score, det_label, gt_box, gt_label = flats
        n_det, n_gt = det_label.shape[0], gt_label.shape[0]
        if (det_box.shape != (n_det, 4) or gt_box.shape != (n_gt, 4) or det_score.shape != (n_det,) or det_label.shape != (n_det,)
                or gt_label.shape != (n_gt,) or (crowd is not None and crowd.shape != (n_gt,)) or (area is not None and area.shape != (n_gt,))
                or len({t.device for t in (*flats, *(c for c in (crowd, area) if c is not None))}) != 1):
            return False
        if crowd is None or area is None:  # absent columns share one zero buffer (read-only state runs)
            zero = torch.zeros_like(gt_label)
            crowd = zero if crowd is None else crowd
            area = zero if area is None else area
        if self.warn_on_many_detections and max(dn) > self.max_detection_thresholds[-1]:
            _warning_on_too_many_detections(self.max_detection_thresholds[-1])
        # lazy runs: the per-image items are views created at their first use (state_dict, list access), not here
        self.detection_box.extend_rows(box_convert(det_box, in_fmt=self.box_format, out_fmt="xywh"), dn, lazy=True)
        self.detection_scores.extend_rows(det_score, dn, lazy=True)
        self.detection_labels.extend_rows(det_label, dn, lazy=True)
        self.groundtruth_box.extend_rows(box_convert(gt_box, in_fmt=self.box_format, out_fmt="xywh"), gn, lazy=True)
        self.groundtruth_labels.extend_rows(gt_label, gn, lazy=True)
        self.groundtruth_crowds.extend_rows(crowd, gn, lazy=True)
        self.groundtruth_area.extend_rows(area, gn, lazy=True)
        return True

    def _convert_boxes(self, boxes: List[Tensor]) -> List[Tensor]:
        """Per-image ``xywh`` boxes; one conversion kernel for the whole batch when the images share device/dtype."""
        boxes = [_fix_empty_tensors(b) for b in boxes]
        uniform = (
            len(boxes) > 1
            and all(b.ndim == 2 and b.shape[-1] == 4 for b in boxes)
            and len({(b.device, b.dtype) for b in boxes}) == 1
        )
        if not uniform:
            out = []
            for b in boxes:
                out.append(box_convert(b, in_fmt=self.box_format, out_fmt="xywh") if b.numel() > 0 else b.reshape(0, 4))
            return out
        sizes = [b.shape[0] for b in boxes]
        flat = torch.cat(boxes)
        if flat.numel() > 0:
            flat = box_convert(flat, in_fmt=self.box_format, out_fmt="xywh")
        return list(torch.split(flat, sizes))

    @staticmethod
    def _optional_column(items: List[Dict[str, Tensor]], key: str, labels: List[Tensor]) -> List[Tensor]:
        """``item[key]`` where present, else zeros shaped like the labels (one shared buffer for the batch)."""
        missing = [i for i, item in enumerate(items) if key not in item]
        out: List[Optional[Tensor]] = [item.get(key) for item in items]
        if missing:
            ref = labels[missing[0]]
            if all(labels[i].device == ref.device and labels[i].dtype == ref.dtype for i in missing):
                sizes = [labels[i].numel() for i in missing]
                zeros = torch.zeros(sum(sizes), dtype=ref.dtype, device=ref.device)
                for i, z in zip(missing, torch.split(zeros, sizes)):
                    out[i] = z.view_as(labels[i])
            else:
                for i in missing:
                    out[i] = torch.zeros_like(labels[i])
        return out  # type: ignore[return-value]

    # ------------------------------------------------------------------------------------------------------
    # evaluation
    # ------------------------------------------------------------------------------------------------------
    def _get_classes(self) -> List:
        if len(self.detection_labels) > 0 or len(self.groundtruth_labels) > 0:
            parts = [
                self._flat_cached(lst, sum(_item_sizes(lst)), torch.long, _first(lst).device)
                for lst in (self.detection_labels, self.groundtruth_labels)
                if len(lst)
            ]
            lab = torch.cat(parts)
            if lab.is_cuda and ops.load():
                # class ids in [0, 65536): a presence bitmap (8 KiB read into pinned memory) and the present ids compacted
                # on the device (tmx::class_presence) instead of torch.unique's sort + size synchronisation
                bm, ids_dev = torch.ops.tmx.class_presence(lab)
                words = bm.numpy().view(np.uint32)
                if not words[-1]:
                    nz = np.flatnonzero(words[:-1])
                    bits = np.unpackbits(words[nz].view(np.uint8), bitorder="little").reshape(-1, 32).view(bool)
                    ids = (nz[:, None] * 32 + np.arange(32))[bits]
                    self.__dict__["_classes_dev"] = ids_dev[: ids.size]
                    return ids.tolist()
            uniq = lab.unique()
            self.__dict__["_classes_dev"] = uniq  # the evaluator's sorted class ids, without a host round trip
            return uniq.cpu().tolist()
        self.__dict__["_classes_dev"] = None
        return []

    _flat_cache: Optional[Dict[Tuple[int, torch.dtype, str, int], Tensor]] = None

    def _flat_cached(self, lst: List[Tensor], n: int, dtype: torch.dtype, dev: torch.device, width: int = 0) -> Tensor:
        """``_flat_rows`` memoised for the duration of one ``compute`` (class discovery and the evaluator flatten the
        same label lists)."""
        cache = self._flat_cache
        if cache is None:
            return _flat_rows(lst, n, dtype, dev, width)
        key = (id(lst), dtype, str(dev), width)
        out = cache.get(key)
        if out is None or out.shape[0] != n:
            out = cache[key] = _flat_rows(lst, n, dtype, dev, width)
        return out

    @staticmethod
    def _flat(lst: List[Tensor], width: Optional[int] = None) -> Tensor:
        if not lst:
            return torch.zeros((0, width) if width else (0,))
        rows = [t.detach().reshape(-1, width) if width else t.detach().reshape(-1) for t in lst]
        return torch.cat([r.cpu() for r in rows])

    def _gpu_eligible(self) -> bool:
        """The device evaluator covers T * A <= 64 (IoU thresholds x 4 area ranges) and up to 256 ascending recall
        thresholds; anything else (and CPU states) takes the host evaluator ``tmx::coco_evaluate``."""
        if not self.groundtruth_labels and not self.detection_labels:
            return False
        sample = _first(self.detection_labels or self.groundtruth_labels)
        if not (sample.is_cuda and ops.use_native(sample)):
            return False
        return self._gpu_eligible_params()

    def _gpu_eligible_params(self) -> bool:
        rt = self.rec_thresholds
        return (
            len(self.iou_thresholds) * len(_AREA_RANGES) <= 64
            and len(rt) <= 256
            and all(rt[i] <= rt[i + 1] for i in range(len(rt) - 1))
        )

    def _evaluate(self, i_type: str, average: str, classes: List[int]) -> _EvalResult:
        if self._gpu_eligible():
            try:
                return self._evaluate_gpu(i_type, average, classes)
            except RuntimeError as err:  # > 1024 ground truths of one class in one image: host evaluator
                if "ground-truth boxes of one class" not in str(err):
                    raise
        return self._evaluate_host(i_type, average, classes)

    _segm_cache: Optional[Tuple[str, Tuple[Tensor, ...]]] = None

    def _segm(self, dev: torch.device) -> Tuple[Tensor, ...]:
        """(flat IoU blocks, per-image offsets, detection mask areas, ground-truth mask areas) from the RLE states,
        computed once per ``compute`` (bbox + segm and class_metrics evaluations reuse it)."""
        key = str(dev)
        if self._segm_cache is None or self._segm_cache[0] != key:
            self._segm_cache = (key, rle_segm_ious(self.detection_mask, self.groundtruth_mask, self.groundtruth_crowds, dev))
        return self._segm_cache[1]

    def _evaluate_gpu(self, i_type: str, average: str, classes: List[int]) -> _EvalResult:
        """Flatten the per-image states on the device and run ``tmx::coco_evaluate_gpu`` (csrc/coco_match.hip):
        matching and accumulation never leave the GPU; one small host read sizes the IoU export."""
        dev = _first(self.detection_labels or self.groundtruth_labels).device
        num_images = len(self.groundtruth_labels)
        det_sizes = _item_sizes(self.detection_labels)
        gt_sizes = _item_sizes(self.groundtruth_labels)
        n_det, n_gt = sum(det_sizes), sum(gt_sizes)

        def flat(lst: List[Tensor], n: int, dtype: torch.dtype, width: int = 0) -> Tensor:
            return self._flat_cached(lst, n, dtype, dev, width)

        cats = self.__dict__.get("_classes_dev")
        if average != "micro" and (cats is None or cats.numel() != len(classes) or cats.device != dev):
            cats = torch.tensor(classes, dtype=torch.long, device=dev)
        if (
            i_type == "bbox" and "segm" not in self.iou_type and not self.extended_summary and _IMG_ROUTE
            and len(det_sizes) == num_images and max(det_sizes, default=0) <= _IMG_ROUTE_ROWS
            and max(gt_sizes, default=0) <= _IMG_ROUTE_ROWS and _score_dtype(self.detection_scores) == torch.float32
        ):
            return self._evaluate_gpu_img(average, classes, cats, det_sizes, gt_sizes, n_det, n_gt, flat)
        det_sz, gt_sz = _h2d_many([det_sizes, gt_sizes], _first(self.detection_labels or self.groundtruth_labels))
        det_img = torch.repeat_interleave(torch.arange(len(det_sizes), device=dev), det_sz, output_size=n_det)
        gt_img = torch.repeat_interleave(torch.arange(num_images, device=dev), gt_sz, output_size=n_gt)
        det_labels = flat(self.detection_labels, n_det, torch.long)
        gt_labels = flat(self.groundtruth_labels, n_gt, torch.long)
        # scores keep an fp32 / 16-bit dtype (the evaluator widens them; fp32-exact scores take its single composite-key
        # radix orderings instead of two stable sorts on doubles)
        det_scores = flat(self.detection_scores, n_det, _score_dtype(self.detection_scores))
        gt_crowd = flat(self.groundtruth_crowds, n_gt, torch.long)
        gt_area = flat(self.groundtruth_area, n_gt, torch.float64)
        if average == "micro":
            cat_ids = [0] if classes else []
            det_cls, gt_cls = torch.zeros_like(det_labels), torch.zeros_like(gt_labels)
        else:
            cat_ids = list(classes)
            det_cls = torch.searchsorted(cats, det_labels)
            gt_cls = torch.searchsorted(cats, gt_labels)

        segm_in = "segm" in self.iou_type
        if segm_in:
            seg_iou, seg_off, det_mask_area, gt_mask_area = self._segm(dev)
        if "bbox" in self.iou_type:
            det_boxes = flat(self.detection_box, n_det, torch.float64, 4)
            gt_boxes = flat(self.groundtruth_box, n_gt, torch.float64, 4)
        else:
            det_boxes = torch.zeros(n_det, 4, dtype=torch.float64, device=dev)
            gt_boxes = torch.zeros(n_gt, 4, dtype=torch.float64, device=dev)
        det_area = det_mask_area if i_type == "segm" else det_boxes[:, 2] * det_boxes[:, 3]
        gt_fallback = gt_mask_area if segm_in else gt_boxes[:, 2] * gt_boxes[:, 3]
        gt_area = torch.where(gt_area > 0, gt_area, gt_fallback)

        img_iou = img_off = det_local = gt_local = img_ng = None
        if i_type == "segm":
            img_iou, img_off = seg_iou, seg_off
            img_ng = gt_sz
            det_first = det_sz.cumsum(0) - det_sz
            gt_first = img_ng.cumsum(0) - img_ng
            det_local = torch.arange(n_det, device=dev) - det_first[det_img]
            gt_local = torch.arange(n_gt, device=dev) - gt_first[gt_img]
            if len(self.iou_type) == 1:
                # the reference's COCO export drops images without ground-truth masks from the evaluated image set
                keep = (img_ng > 0)[det_img]
                det_boxes, det_scores, det_cls, det_area = det_boxes[keep], det_scores[keep], det_cls[keep], det_area[keep]
                det_img, det_local = det_img[keep], det_local[keep]

        prec, rec, _scores, iou_values, iou_index, overflow = torch.ops.tmx.coco_evaluate_gpu(
            det_boxes, det_scores, det_cls, det_img, det_area, gt_boxes, gt_cls, gt_img, gt_crowd, gt_area,
            len(cat_ids), num_images, *self._eval_params(dev),
            img_iou, img_off, det_local, gt_local, img_ng, self.extended_summary,
        )
        # precision / recall stay on the device (summarised there, copied only for extended_summary); the IoU export
        # exists only for extended_summary (empty otherwise: no copy)
        if self.extended_summary:
            iou_values, iou_index = iou_values.cpu(), iou_index.cpu()
        return _EvalResult(prec, rec, iou_values, iou_index, cat_ids, num_images, overflow)

    def _evaluate_gpu_img(self, average: str, classes: List[int], cats: Optional[Tensor], det_sizes: List[int],
                          gt_sizes: List[int], n_det: int, n_gt: int, flat: Any) -> _EvalResult:
        """bbox evaluation on the per-image route (``tmx::coco_evaluate_gpu_img``): one workgroup per image orders,
        ranks and matches its own rows, so no global sort by (image, class), no (image, class) grid lookups and no
        row gathers run before the accumulate step; the image offsets come from the host-held item sizes."""
        like = _first(self.detection_labels or self.groundtruth_labels)
        nd1 = len(det_sizes) + 1
        off = np.fromiter(itertools.chain((0,), det_sizes, (0,), gt_sizes), dtype=np.int64, count=nd1 + len(gt_sizes) + 1)
        np.cumsum(off[:nd1], out=off[:nd1])
        np.cumsum(off[nd1:], out=off[nd1:])
        off_t = torch.from_numpy(off)
        off_t = torch.ops.tmx.upload_i64(off_t, like) if like.is_cuda and ops.load() else off_t.to(like.device)
        det_labels = flat(self.detection_labels, n_det, torch.long)
        gt_labels = flat(self.groundtruth_labels, n_gt, torch.long)
        det_scores = flat(self.detection_scores, n_det, torch.float32)
        gt_crowd = flat(self.groundtruth_crowds, n_gt, torch.long)
        gt_area = flat(self.groundtruth_area, n_gt, torch.float64)
        det_boxes = flat(self.detection_box, n_det, torch.float64, 4)
        gt_boxes = flat(self.groundtruth_box, n_gt, torch.float64, 4)
        if average == "micro":
            cat_ids = [0] if classes else []
            det_cls, gt_cls = torch.zeros_like(det_labels), torch.zeros_like(gt_labels)
        else:
            cat_ids = list(classes)
            det_cls = torch.searchsorted(cats, det_labels)
            gt_cls = torch.searchsorted(cats, gt_labels)
        # (areas: the kernel takes box areas for detections and the supplied ground-truth area where > 0, else the box's)
        iou_thr, rec_thr, max_dets, area_rng = self._eval_params(det_scores.device)
        prec, rec, _scores, overflow = torch.ops.tmx.coco_evaluate_gpu_img(
            det_boxes, det_scores, det_cls, off_t[:nd1], gt_boxes, gt_cls, gt_crowd, gt_area, off_t[nd1:],
            len(cat_ids), iou_thr, rec_thr, max_dets, self._param_cache[2], area_rng,
        )
        empty = torch.zeros(0, dtype=torch.float64)
        return _EvalResult(prec, rec, empty, torch.zeros(0, 5, dtype=torch.long), cat_ids, len(gt_sizes), overflow)

    _param_cache: Optional[Tuple[Any, Tuple[Tensor, ...]]] = None

    def _eval_params(self, dev: torch.device) -> Tuple[Tensor, ...]:
        """(IoU thresholds, recall thresholds, max detections (host), area ranges) as evaluator inputs, built once per
        device and threshold set (four small host->device copies per compute otherwise)."""
        key = (str(dev), tuple(self.iou_thresholds), tuple(self.rec_thresholds), tuple(self.max_detection_thresholds))
        cached = self._param_cache
        if cached is None or cached[0] != key:
            md = torch.tensor(self.max_detection_thresholds, dtype=torch.long)
            cached = self._param_cache = (key, (
                torch.tensor(self.iou_thresholds, dtype=torch.float64, device=dev),
                torch.tensor(self.rec_thresholds, dtype=torch.float64, device=dev),
                md,
                torch.tensor(_AREA_RANGES, dtype=torch.float64, device=dev),
            ), md.to(dev))  # (+ a device copy of the thresholds for the per-image route)
        return cached[1]

    def _evaluate_host(self, i_type: str, average: str, classes: List[int]) -> _EvalResult:
        num_images = len(self.groundtruth_labels)
        det_counts = torch.tensor([t.numel() for t in self.detection_labels], dtype=torch.long)
        gt_counts = torch.tensor([t.numel() for t in self.groundtruth_labels], dtype=torch.long)
        det_img = torch.repeat_interleave(torch.arange(len(self.detection_labels)), det_counts)
        gt_img = torch.repeat_interleave(torch.arange(num_images), gt_counts)
        det_labels = self._flat(self.detection_labels).long()
        gt_labels = self._flat(self.groundtruth_labels).long()
        det_scores = self._flat(self.detection_scores).double()
        gt_crowd = self._flat(self.groundtruth_crowds).long()
        gt_area = self._flat(self.groundtruth_area).double()
        if average == "micro":
            det_labels, gt_labels = torch.zeros_like(det_labels), torch.zeros_like(gt_labels)
            cat_ids = [0] if classes else []
        else:
            cat_ids = list(classes)

        segm_in = "segm" in self.iou_type
        if segm_in:
            seg_iou, seg_off, det_mask_area, gt_mask_area = (t.cpu() for t in self._segm(torch.device("cpu")))
        if "bbox" in self.iou_type:
            det_boxes = self._flat(self.detection_box, 4).double()
            gt_boxes = self._flat(self.groundtruth_box, 4).double()
        else:
            det_boxes = torch.zeros(det_labels.numel(), 4, dtype=torch.float64)
            gt_boxes = torch.zeros(gt_labels.numel(), 4, dtype=torch.float64)

        # areas: detections use the area of the evaluated representation; ground truth uses the supplied area when
        # positive, else the mask area whenever masks are tracked (box area otherwise) - as the reference's COCO export
        det_area = det_mask_area if i_type == "segm" else det_boxes[:, 2] * det_boxes[:, 3]
        gt_fallback = gt_mask_area if segm_in else gt_boxes[:, 2] * gt_boxes[:, 3]
        gt_area = torch.where(gt_area > 0, gt_area, gt_fallback)

        img_iou = img_off = None
        if i_type == "segm":
            img_iou, img_off = seg_iou, seg_off
            if len(self.iou_type) == 1:
                # the reference's COCO export drops images without ground-truth masks from the evaluated image set
                keep_img = gt_counts > 0
                keep = keep_img[det_img] if det_img.numel() else torch.zeros(0, dtype=torch.bool)
                det_boxes, det_scores, det_labels, det_area = det_boxes[keep], det_scores[keep], det_labels[keep], det_area[keep]
                det_img_kept = det_img[keep]
                # custom IoU matrices index detections by their row within the image: keep rows contiguous by
                # only dropping whole images (all of an image's rows go, or none)
                det_img = det_img_kept

        prec, rec, _scores, iou_values, iou_index = torch.ops.tmx.coco_evaluate(
            det_boxes, det_scores, det_labels, det_img, det_area,
            gt_boxes, gt_labels, gt_img, gt_crowd, gt_area,
            torch.tensor(cat_ids, dtype=torch.long), num_images,
            torch.tensor(self.iou_thresholds, dtype=torch.float64),
            torch.tensor(self.rec_thresholds, dtype=torch.float64),
            torch.tensor(self.max_detection_thresholds, dtype=torch.long),
            torch.tensor(_AREA_RANGES, dtype=torch.float64),
            img_iou, img_off,
        )
        return _EvalResult(prec, rec, iou_values, iou_index, cat_ids, num_images)

    # ------------------------------------------------------------------------------------------------------
    # class-sharded compute (``sharded_compute=True`` under DDP; boxes, macro average)
    # ------------------------------------------------------------------------------------------------------
    # The reference gathers every image's boxes to every rank and each rank evaluates every class
    # (``mean_ap.py:501-575``).  Here rows are routed to the rank owning their class (class index mod world) with one
    # all_to_all per column (parallel/shard.py); each rank matches and accumulates only its classes (the other
    # classes have no rows there and stay -1), and one MAX all-reduce of the precision / recall tables assembles the
    # full result on every rank.  Image ids are made global in the replicated gather's (rank-interleaved) order.
    _shard_flat: Optional[Dict[str, Any]] = None

    def _shardable(self, dist_sync_fn: Any) -> bool:
        from torchmetrics_forked_amd.utilities.distributed import gather_all_tensors

        return (
            self.sharded_compute and self.iou_type == ("bbox",) and self.average == "macro" and not self.extended_summary
            and (dist_sync_fn is None or dist_sync_fn is gather_all_tensors)
        )

    def _local_bbox_rows(self, dev: torch.device) -> Dict[str, Tensor]:
        det_sizes = [t.numel() for t in self.detection_labels]
        gt_sizes = [t.numel() for t in self.groundtruth_labels]

        def flat(lst: List[Tensor], n: int, dtype: torch.dtype, width: int = 0) -> Tensor:
            return _flat_rows(lst, n, dtype, dev, width)

        n_det, n_gt = sum(det_sizes), sum(gt_sizes)
        return {
            "det_boxes": flat(self.detection_box, n_det, torch.float64, 4),
            "det_scores": flat(self.detection_scores, n_det, torch.float64),
            "det_labels": flat(self.detection_labels, n_det, torch.long),
            "det_img": torch.repeat_interleave(torch.arange(len(det_sizes), device=dev), torch.tensor(det_sizes, dtype=torch.long, device=dev),
                                               output_size=n_det),
            "gt_boxes": flat(self.groundtruth_box, n_gt, torch.float64, 4),
            "gt_labels": flat(self.groundtruth_labels, n_gt, torch.long),
            "gt_img": torch.repeat_interleave(torch.arange(len(gt_sizes), device=dev), torch.tensor(gt_sizes, dtype=torch.long, device=dev),
                                              output_size=n_gt),
            "gt_crowd": flat(self.groundtruth_crowds, n_gt, torch.long),
            "gt_area": flat(self.groundtruth_area, n_gt, torch.float64),
        }

    def _sync_dist(self, dist_sync_fn: Any = None, process_group: Optional[Any] = None) -> None:
        if not self._shardable(dist_sync_fn):
            if "segm" in self.iou_type:
                # RLE tuples ride the packed all-gather as one uint8 tensor per image (same element-major,
                # rank-interleaved order as every other list state; the reference uses all_gather_object)
                self.detection_mask = _pack_rle_states(self.detection_mask, self.device)
                self.groundtruth_mask = _pack_rle_states(self.groundtruth_mask, self.device)
            super()._sync_dist(dist_sync_fn, process_group)
            if "segm" in self.iou_type:
                self.detection_mask = _unpack_rle_states(self.detection_mask)
                self.groundtruth_mask = _unpack_rle_states(self.groundtruth_mask)
            return
        import torch.distributed as dist

        from torchmetrics_forked_amd.parallel.shard import exchange_rows
        from torchmetrics_forked_amd.parallel.sync import _collective, _comm_device
        from torchmetrics_forked_amd.utilities.distributed import gather_all_tensors

        group = process_group or self.process_group
        world = dist.get_world_size(group) if group is not None else dist.get_world_size()
        rank = dist.get_rank(group) if group is not None else dist.get_rank()
        dev = self.device
        rows = self._local_bbox_rows(dev)
        cdev = _comm_device(rows["det_scores"], group)
        n_img = torch.tensor([len(self.groundtruth_labels)], dtype=torch.long, device=cdev)
        all_n = torch.empty(world, dtype=torch.long, device=cdev)
        _collective(dist.all_gather_into_tensor, all_n, n_img, what="all_gather(image counts)", group=group)
        counts = all_n.tolist()
        # global image ids in the order of the replicated sync (and of the reference's gather): element-major,
        # rank-interleaved - image e of rank r sits after every rank's images < e and lower ranks' image e
        cnt = torch.tensor(counts, dtype=torch.long, device=dev)
        e = torch.arange(len(self.groundtruth_labels), dtype=torch.long, device=dev)
        gid = torch.minimum(cnt[None, :], e[:, None]).sum(1) + (cnt[None, :rank] > e[:, None]).sum(1)
        local_cls = torch.cat([rows["det_labels"], rows["gt_labels"]]).unique().to(cdev)
        classes = torch.cat([t.to(cdev) for t in gather_all_tensors(local_cls, group)]).unique().to(dev)
        owner_of = lambda lab: torch.searchsorted(classes, lab).remainder(world)  # noqa: E731
        det, _ = exchange_rows(
            [rows["det_boxes"], rows["det_scores"], rows["det_labels"], gid[rows["det_img"]]], owner_of(rows["det_labels"]), group
        )
        gt, _ = exchange_rows(
            [rows["gt_boxes"], rows["gt_labels"], gid[rows["gt_img"]], rows["gt_crowd"], rows["gt_area"]], owner_of(rows["gt_labels"]), group
        )
        self._shard_flat = {
            "det_boxes": det[0].to(dev).reshape(-1, 4), "det_scores": det[1].to(dev), "det_labels": det[2].to(dev), "det_img": det[3].to(dev),
            "gt_boxes": gt[0].to(dev).reshape(-1, 4), "gt_labels": gt[1].to(dev), "gt_img": gt[2].to(dev), "gt_crowd": gt[3].to(dev),
            "gt_area": gt[4].to(dev), "num_images": sum(counts), "classes": classes.cpu().tolist(), "group": group,
        }

    def unsync(self, should_unsync: bool = True) -> None:
        super().unsync(should_unsync)
        if should_unsync:
            self._shard_flat = None

    def sync(self, dist_sync_fn: Any = None, process_group: Optional[Any] = None, should_sync: bool = True,
             distributed_available: Optional[Any] = None, async_op: bool = False) -> Any:
        """RLE mask states are packed around the blocking sync (``_sync_dist``); ``async_op`` therefore completes the
        sync before returning an already-finished handle when masks are tracked."""
        if async_op and "segm" in self.iou_type:
            from torchmetrics_forked_amd.metric import _MetricPendingSync

            super().sync(dist_sync_fn, process_group, should_sync, distributed_available, async_op=False)
            return _MetricPendingSync(self, None)
        return super().sync(dist_sync_fn, process_group, should_sync, distributed_available, async_op=async_op)

    def _evaluate_sharded(self, classes: List[int]) -> _EvalResult:
        """This rank's classes from the exchanged rows, then MAX all-reduce of the tables (-1 = not evaluated here)."""
        from torchmetrics_forked_amd.parallel.shard import all_reduce_max

        f = self._shard_flat
        dev = f["det_scores"].device
        gt_area = torch.where(f["gt_area"] > 0, f["gt_area"], f["gt_boxes"][:, 2] * f["gt_boxes"][:, 3])
        det_area = f["det_boxes"][:, 2] * f["det_boxes"][:, 3]
        args = (
            torch.tensor(self.iou_thresholds, dtype=torch.float64, device=dev),
            torch.tensor(self.rec_thresholds, dtype=torch.float64, device=dev),
            torch.tensor(self.max_detection_thresholds, dtype=torch.long),
            torch.tensor(_AREA_RANGES, dtype=torch.float64, device=dev),
        )
        cats = torch.tensor(classes, dtype=torch.long, device=dev)
        gpu_ok = dev.type == "cuda" and ops.use_native(f["det_scores"]) and self._gpu_eligible_params()
        if gpu_ok:
            prec, rec, _, _, _, overflow = torch.ops.tmx.coco_evaluate_gpu(
                f["det_boxes"], f["det_scores"], torch.searchsorted(cats, f["det_labels"]), f["det_img"], det_area,
                f["gt_boxes"], torch.searchsorted(cats, f["gt_labels"]), f["gt_img"], f["gt_crowd"], gt_area,
                len(classes), f["num_images"], *args, None, None, None, None, None, False,
            )
            gpu_ok = not bool(overflow.item())  # (this path reads its tables on the host below anyway)
        if not gpu_ok:
            prec, rec, _, _, _ = torch.ops.tmx.coco_evaluate(
                f["det_boxes"].cpu(), f["det_scores"].cpu(), f["det_labels"].cpu(), f["det_img"].cpu(), det_area.cpu(),
                f["gt_boxes"].cpu(), f["gt_labels"].cpu(), f["gt_img"].cpu(), f["gt_crowd"].cpu(), gt_area.cpu(),
                cats.cpu(), f["num_images"], *[a.cpu() for a in args], None, None,
            )
        prec = all_reduce_max(prec.to(dev), f["group"]).cpu()
        rec = all_reduce_max(rec.to(dev), f["group"]).cpu()
        empty = torch.zeros(0)
        return _EvalResult(prec, rec, empty, torch.zeros(0, 5, dtype=torch.long), list(classes), f["num_images"])

    def _summary_tables(self, precision: Tensor, recall: Tensor, overflow: Optional[Tensor] = None) -> Optional[np.ndarray]:
        """Sums and counts of the valid (``> -1``) entries of ``precision [T,R,K,A,M]`` (summed over R) and ``recall
        [T,K,A,M]``, as one host array ``[4, T, K, A, M]``: a few reductions where the tables live (the device, for the
        GPU evaluator) and ONE small copy, instead of copying both tables and slicing them twelve times per summary."""
        if precision.is_cuda and precision.dim() == 5 and ops.load():  # one kernel + one pinned copy (tmx::coco_summary_tables)
            both = torch.ops.tmx.coco_summary_tables(precision, recall, overflow).numpy()
            if both[-1] != 0:
                return None
            t, _, k, a, m = precision.shape
            return both[:-1].reshape(4, t, k, a, m)
        vp = precision > -1
        vr = recall > -1
        tab = torch.stack([
            torch.where(vp, precision, 0.0).sum(1, dtype=torch.float64), vp.sum(1, dtype=torch.float64),
            torch.where(vr, recall, 0.0).to(torch.float64), vr.to(torch.float64),
        ])
        if overflow is None:
            return tab.cpu().numpy()
        # the GPU evaluator's overflow flag travels in the same copy; None = the tables are invalid
        both = torch.cat([tab.reshape(-1), overflow.to(torch.float64).reshape(-1)]).cpu().numpy()
        return None if both[-1] != 0 else both[:-1].reshape(tab.shape)

    def _summarize_tables(self, tab: np.ndarray, k: Optional[int] = None) -> List[float]:
        """COCO ``summarize()`` statistics (all classes, or class index ``k``) from ``_summary_tables``: each statistic
        is the mean of the valid entries it selects (-1 when there are none)."""
        md = self.max_detection_thresholds
        thr = self.iou_thresholds
        if k is not None:
            tab = tab[:, :, k : k + 1]

        def stat(ap: bool, iou: Optional[float] = None, area: int = 0, max_det: int = 100) -> float:
            mind = [i for i, m in enumerate(md) if m == max_det]
            tsel = [i for i, v in enumerate(thr) if v == iou] if iou is not None else None
            base = 0 if ap else 2
            if len(mind) == 1 and (tsel is None or len(tsel) == 1):  # basic indexing: views, no fancy-index copies
                sub = tab[base : base + 2, slice(None) if tsel is None else tsel[0], :, area, mind[0]]
            else:
                sub = tab[base : base + 2][:, list(range(len(thr))) if tsel is None else tsel][:, :, :, area][..., mind]
            total, count = float(sub[0].sum()), float(sub[1].sum())
            return total / count if count > 0 else -1.0

        last = md[2] if len(md) > 2 else md[-1]
        first_map = 100 if self.backend == "pycocotools" else md[-1]
        return [
            stat(True, max_det=first_map),
            stat(True, iou=0.5, max_det=last),
            stat(True, iou=0.75, max_det=last),
            stat(True, area=1, max_det=last),
            stat(True, area=2, max_det=last),
            stat(True, area=3, max_det=last),
            stat(False, max_det=md[0]),
            stat(False, max_det=md[1] if len(md) > 1 else md[-1]),
            stat(False, max_det=last),
            stat(False, area=1, max_det=last),
            stat(False, area=2, max_det=last),
            stat(False, area=3, max_det=last),
        ]

    def _per_class_stats(self, tab: np.ndarray) -> Tuple[Tensor, Tensor]:
        """``map`` (stats[0]) and ``mar_100`` (stats[8]) of every class at once from ``_summary_tables``: the same
        selections as ``_summarize_tables(tab, k)`` reduced over the IoU thresholds / maxDets axes for all classes in two
        numpy reductions each, instead of twelve statistics per class in a Python loop (10 ms at 80 classes)."""
        md = self.max_detection_thresholds
        last = md[2] if len(md) > 2 else md[-1]
        first_map = 100 if self.backend == "pycocotools" else md[-1]

        def per_class(base: int, max_det: int) -> Tensor:
            mind = [i for i, m in enumerate(md) if m == max_det]
            sub = tab[base : base + 2, :, :, 0][..., mind]  # [2, T, K, len(mind)]
            total, count = sub[0].sum(axis=(0, 2)), sub[1].sum(axis=(0, 2))
            with np.errstate(divide="ignore", invalid="ignore"):
                val = np.where(count > 0, total / np.where(count > 0, count, 1.0), -1.0)
            return torch.from_numpy(val.astype(np.float32))

        return per_class(0, first_map), per_class(2, last)

    def _summarize(self, precision: Tensor, recall: Tensor) -> List[float]:
        """COCO ``summarize()`` statistics from accumulated ``precision [T,R,K,A,M]`` / ``recall [T,K,A,M]``."""
        return self._summarize_tables(self._summary_tables(precision, recall))

    @staticmethod
    def _coco_stats_to_tensor_dict(stats: List[float], prefix: str) -> Dict[str, Tensor]:
        # one host tensor, twelve [1]-element views (one allocation instead of twelve)
        return dict(zip((f"{prefix}{n}" for n in _STAT_NAMES), torch.tensor(stats, dtype=torch.float32).split(1)))

    def _ious_dict(self, ev: _EvalResult) -> Dict[Tuple[int, int], Any]:
        """Every (image, category) pair in pycocotools' order; pairs without both detections and ground truth
        map to ``[]``."""
        out: Dict[Tuple[int, int], Any] = {(i, c): [] for i in range(ev.num_images) for c in ev.cat_ids}
        vals = ev.iou_values
        for img, k, nd, ng, off in ev.iou_index.tolist():
            if nd and ng:
                out[(img, ev.cat_ids[k])] = vals[off : off + nd * ng].reshape(nd, ng).float()
        return out

    def compute(self) -> dict:
        ops.require()
        self._segm_cache = None
        self._flat_cache = {}
        try:
            return self._compute()
        finally:
            self._segm_cache = None
            self._flat_cache = None
            self.__dict__["_classes_dev"] = None

    def _compute(self) -> dict:
        sharded = self._shard_flat is not None
        classes = self._shard_flat["classes"] if sharded else self._get_classes()
        result: Dict[str, Any] = {}
        for i_type in self.iou_type:
            prefix = "" if len(self.iou_type) == 1 else f"{i_type}_"
            ev = self._evaluate_sharded(classes) if sharded else self._evaluate(i_type, self.average, classes)
            tab = self._summary_tables(ev.precision, ev.recall, ev.overflow)
            if tab is None:  # > 1024 ground truths of one class in one image: the host evaluator
                ev = self._evaluate_host(i_type, self.average, classes)
                tab = self._summary_tables(ev.precision, ev.recall)
            result.update(self._coco_stats_to_tensor_dict(self._summarize_tables(tab), prefix))
            if self.extended_summary:
                result[f"{prefix}ious"] = self._ious_dict(ev)
                result[f"{prefix}precision"] = ev.precision.cpu()
                result[f"{prefix}recall"] = ev.recall.cpu()
            if self.class_metrics:
                if self.average == "micro":
                    ev = self._evaluate(i_type, "macro", classes)
                    tab = self._summary_tables(ev.precision, ev.recall, ev.overflow)
                    if tab is None:
                        ev = self._evaluate_host(i_type, "macro", classes)
                        tab = self._summary_tables(ev.precision, ev.recall)
                map_pc_t, mar_pc_t = self._per_class_stats(tab)
            else:
                map_pc_t = torch.tensor([-1], dtype=torch.float32)
                mar_pc_t = torch.tensor([-1], dtype=torch.float32)
            result[f"{prefix}map_per_class"] = map_pc_t
            result[f"{prefix}mar_100_per_class"] = mar_pc_t
        result["classes"] = torch.tensor(classes, dtype=torch.int32)
        return result

    # ------------------------------------------------------------------------------------------------------
    # COCO json interop
    # ------------------------------------------------------------------------------------------------------
    @staticmethod
    def coco_to_tm(
        coco_preds: str,
        coco_target: str,
        iou_type: Union[Literal["bbox", "segm"], List[str]] = "bbox",
        backend: Literal["pycocotools", "faster_coco_eval"] = "pycocotools",
    ) -> Tuple[List[Dict[str, Tensor]], List[Dict[str, Tensor]]]:
        """Read COCO-format json files (ground-truth dataset + result list) into this metric's input format.

        Boxes stay in COCO ``xywh``; masks are decoded from polygons / RLE.  Only images that carry ground-truth
        annotations are returned (reference ``mean_ap.py:628-737``)."""
        iou_type = _validate_iou_type_arg(iou_type)
        with open(coco_target) as f:
            gt_ds = json.load(f)
        with open(coco_preds) as f:
            dt = json.load(f)
        dt_anns = dt["annotations"] if isinstance(dt, dict) else dt
        img_hw = {im["id"]: (im.get("height"), im.get("width")) for im in gt_ds.get("images", [])}

        def mask_of(ann: Dict[str, Any]) -> np.ndarray:
            h, w = img_hw[ann["image_id"]]
            return segmentation_to_mask(ann["segmentation"], h, w)

        target: Dict[int, Dict[str, list]] = {}
        for t in gt_ds["annotations"]:
            entry = target.setdefault(t["image_id"], {"labels": [], "iscrowd": [], "area": [], "boxes": [], "masks": []})
            if "bbox" in iou_type:
                entry["boxes"].append(t["bbox"])
            if "segm" in iou_type:
                entry["masks"].append(mask_of(t))
            entry["labels"].append(t["category_id"])
            entry["iscrowd"].append(t.get("iscrowd", 0))
            entry["area"].append(t["area"])
        preds: Dict[int, Dict[str, list]] = {}
        for p in dt_anns:
            entry = preds.setdefault(p["image_id"], {"scores": [], "labels": [], "boxes": [], "masks": []})
            if "bbox" in iou_type:
                box = p.get("bbox")
                if box is None:  # segmentation results: bbox derived from the mask
                    m = mask_of(p)
                    ys, xs = np.nonzero(m)
                    box = [float(xs.min()), float(ys.min()), float(xs.max() - xs.min() + 1), float(ys.max() - ys.min() + 1)] \
                        if xs.size else [0.0, 0.0, 0.0, 0.0]
                entry["boxes"].append(box)
            if "segm" in iou_type:
                entry["masks"].append(mask_of(p))
            entry["scores"].append(p["score"])
            entry["labels"].append(p["category_id"])

        batched_preds, batched_target = [], []
        for key, t in target.items():
            p = preds.get(key, {"scores": [], "labels": [], "boxes": [], "masks": []})
            bp = {
                "scores": torch.tensor(p["scores"], dtype=torch.float32),
                "labels": torch.tensor(p["labels"], dtype=torch.int32),
            }
            bt = {
                "labels": torch.tensor(t["labels"], dtype=torch.int32),
                "iscrowd": torch.tensor(t["iscrowd"], dtype=torch.int32),
                "area": torch.tensor(t["area"], dtype=torch.float32),
            }
            if "bbox" in iou_type:
                bp["boxes"] = torch.tensor(np.array(p["boxes"], dtype=np.float32).reshape(-1, 4))
                bt["boxes"] = torch.tensor(np.array(t["boxes"], dtype=np.float32).reshape(-1, 4))
            if "segm" in iou_type:
                bp["masks"] = torch.tensor(np.array(p["masks"]), dtype=torch.uint8)
                bt["masks"] = torch.tensor(np.array(t["masks"]), dtype=torch.uint8)
            batched_preds.append(bp)
            batched_target.append(bt)
        return batched_preds, batched_target

    def _coco_dataset(self, detections: bool) -> Dict[str, Any]:
        labels = self.detection_labels if detections else self.groundtruth_labels
        boxes = self.detection_box if detections else self.groundtruth_box
        masks = self.detection_mask if detections else self.groundtruth_mask
        images, annotations = [], []
        ann_id = 1
        for img_id, lab in enumerate(labels):
            images.append({"id": img_id})
            lab_l = lab.cpu().tolist()
            box_l = boxes[img_id].cpu().tolist() if "bbox" in self.iou_type else None
            msk = masks[img_id] if "segm" in self.iou_type else None
            if msk:
                images[-1]["height"], images[-1]["width"] = int(msk[0][0][0]), int(msk[0][0][1])
            for k, label in enumerate(lab_l):
                ann: Dict[str, Any] = {"id": ann_id, "image_id": img_id, "category_id": int(label)}
                rle = {"size": list(msk[k][0]), "counts": msk[k][1].decode("ascii")} if msk else None
                if detections:
                    ann["score"] = float(self.detection_scores[img_id][k])
                    ann["iscrowd"] = 0
                    area = None
                else:
                    ann["iscrowd"] = int(self.groundtruth_crowds[img_id][k])
                    area = float(self.groundtruth_area[img_id][k])
                if area is None or area <= 0:
                    area = float(rle_state_area(msk[k])) if rle is not None else float(box_l[k][2] * box_l[k][3])
                ann["area"] = area
                if box_l is not None:
                    ann["bbox"] = box_l[k]
                if rle is not None:
                    ann["segmentation"] = rle
                annotations.append(ann)
                ann_id += 1
        cats = [{"id": i, "name": str(i)} for i in self._get_classes()]
        return {"images": images, "annotations": annotations, "categories": cats}

    def tm_to_coco(self, name: str = "tm_map_input") -> None:
        """Write the cached inputs as COCO json: ``{name}_preds.json`` (result list) and ``{name}_target.json``."""
        preds = self._coco_dataset(detections=True)
        target = self._coco_dataset(detections=False)
        with open(f"{name}_preds.json", "w") as f:
            f.write(json.dumps(preds["annotations"], indent=4))
        with open(f"{name}_target.json", "w") as f:
            f.write(json.dumps(target, indent=4))

    def plot(
        self, val: Optional[Union[Dict[str, Tensor], Sequence[Dict[str, Tensor]]]] = None, ax: Optional[_AX_TYPE] = None
    ) -> _PLOT_OUT_TYPE:
        return self._plot(val, ax)


def _flat_rows(lst: List[Tensor], n: int, dtype: torch.dtype, dev: torch.device, width: int = 0) -> Tensor:
    """Concatenate per-image state tensors into one ``[n]`` / ``[n, width]`` tensor.  The states already have that
    layout (update stores ``[k]`` / ``[k, 4]`` per image), so the list goes to ``torch.cat`` as is: a per-element
    ``reshape`` costs more host time than the copy itself at 10k images; only irregular lists take that path."""
    if not lst:
        return torch.zeros((n, width) if width else (n,), dtype=dtype, device=dev)
    try:
        pieces = lst.pieces() if isinstance(lst, StateArena) else lst  # one piece per update batch when recorded
        out = pieces[0] if len(pieces) == 1 else torch.cat(pieces)
        if out.shape != ((n, width) if width else (n,)):
            raise RuntimeError("irregular")
    except RuntimeError:
        out = torch.cat([t.reshape(-1, width) if width else t.reshape(-1) for t in lst])
    return out.to(dev, dtype)


_BOXES, _SCORES, _LABELS = operator.itemgetter("boxes"), operator.itemgetter("scores"), operator.itemgetter("labels")


_CLASS_MAP = 1 << 16  # class ids below this are found with a presence map (_get_classes)
# bbox evaluation on the per-image route (tmx::coco_evaluate_gpu_img) when every image holds at most this many
# detections and ground truths; TMX_MAP_IMG_ROUTE=0 keeps the (image, class)-grid evaluator
_IMG_ROUTE_ROWS = 256
_IMG_ROUTE = os.environ.get("TMX_MAP_IMG_ROUTE", "1") != "0"
_PRED_KEYS, _PRED_WIDTHS = ("boxes", "scores", "labels"), (4, 0, 0)
_GT_KEYS, _GT_WIDTHS = ("boxes", "labels", "iscrowd", "area"), (4, 0, -1, -1)  # (-1: optional 1-d column)


def _optional_col(items: List[Dict[str, Tensor]], key: str) -> Optional[List[Tensor]]:
    """``key`` of every item, ``None`` when no item has it; raises ``KeyError`` when only some do (the batched update
    then leaves the batch to the per-image path)."""
    try:
        return list(map(operator.itemgetter(key), items))
    except KeyError:
        if any(map(operator.contains, items, itertools.repeat(key))):
            raise
        return None


def _score_dtype(lst: List[Tensor]) -> torch.dtype:
    """fp32 when every stored score tensor is fp32 / fp16 / bf16 (exact in fp32), else fp64."""
    pieces = lst.pieces() if isinstance(lst, StateArena) else lst
    low = (torch.float32, torch.float16, torch.bfloat16)
    return torch.float32 if pieces and all(t.dtype in low for t in pieces) else torch.float64


def _item_sizes(lst: List[Tensor]) -> List[int]:
    """``numel`` of every per-image item (the arena's run records when it has them: no per-item tensor call)."""
    if isinstance(lst, StateArena) and lst._runs is not None and (not lst._runs or lst._runs[0][0].ndim == 1):
        return lst.item_rows()
    return [t.numel() for t in lst]


def _first(lst: List[Tensor]) -> Tensor:
    """The first per-image item's tensor (a run of a lazy arena: same device and dtype, no item materialised)."""
    return lst.first_piece() if isinstance(lst, StateArena) else lst[0]


def _pack_rle_states(states: List[Tuple[Tuple[Tuple[int, int], bytes], ...]], device: torch.device) -> List[Tensor]:
    """Per image: one uint8 tensor ``[n, (h, w, len) x n]`` (int64 little endian) + the concatenated counts, built
    as ONE host buffer moved to ``device`` once and split into per-image views."""
    parts: List[bytes] = []
    sizes: List[int] = []
    for entry in states:
        head = np.empty(1 + 3 * len(entry), dtype="<i8")
        head[0] = len(entry)
        for j, ((h, w), counts) in enumerate(entry):
            head[1 + 3 * j: 4 + 3 * j] = (h, w, len(counts))
        blob = head.tobytes() + b"".join(c for _, c in entry)
        parts.append(blob)
        sizes.append(len(blob))
    if not parts:
        return []
    flat = torch.frombuffer(bytearray(b"".join(parts)), dtype=torch.uint8).to(device)
    return list(torch.split(flat, sizes))


def _unpack_rle_states(packed: List[Tensor]) -> List[Tuple[Tuple[Tuple[int, int], bytes], ...]]:
    if not packed:
        return []
    sizes = [int(t.numel()) for t in packed]
    buf = torch.cat([t.reshape(-1) for t in packed]).cpu().numpy().tobytes()
    out: List[Tuple[Tuple[Tuple[int, int], bytes], ...]] = []
    pos = 0
    for size in sizes:
        n = int(np.frombuffer(buf, dtype="<i8", count=1, offset=pos)[0])
        head = np.frombuffer(buf, dtype="<i8", count=3 * n, offset=pos + 8).reshape(n, 3)
        p = pos + 8 * (1 + 3 * n)
        entry = []
        for h, w, ln in head.tolist():
            entry.append(((int(h), int(w)), buf[p:p + ln]))
            p += ln
        out.append(tuple(entry))
        pos += size
    return out


def _warning_on_too_many_detections(limit: int) -> None:
    rank_zero_warn(
        f"Encountered more than {limit} detections in a single image. This means that certain detections with the"
        " lowest scores will be ignored, that may have an undesirable impact on performance. Please consider adjusting"
        " the `max_detection_threshold` to suit your use case. To disable this warning, set attribute class"
        " `warn_on_many_detections=False`, after initializing the metric.",
        UserWarning,
    )
