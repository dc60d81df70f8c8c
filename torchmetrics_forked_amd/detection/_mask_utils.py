"""Segmentation-mask utilities for detection metrics (no pycocotools dependency).

* COCO run-length encoding: column-major runs starting with a background run, compressed to the COCO
  "counts" string (6-bit chunks, ``+48``, differences against the run two places back for runs > 2).
* Polygon rasterisation with the COCO boundary-walk algorithm (×5 upsampled boundary, y-boundary crossings,
  run construction) so masks decoded from polygon annotations match the official tools pixel for pixel.
* ``mask_iou``: pairwise mask IoU.  On GPU masks are bit-packed 64 pixels per word and intersected with the
  ``tmx::mask_iou`` popcount kernel; on CPU a float matmul of the flattened masks (exact integer counts).
"""
from typing import Any, Dict, List, Sequence, Tuple, Union

import math

import numpy as np
import torch
from torch import Tensor

from torchmetrics_forked_amd import ops


# ------------------------------------------------------------------------------------------------------------
# run-length encoding
# ------------------------------------------------------------------------------------------------------------
def _runs(mask: np.ndarray) -> List[int]:
    flat = np.asarray(mask, dtype=np.uint8).reshape(-1, order="F")
    if flat.size == 0:
        return [0]
    change = np.flatnonzero(flat[1:] != flat[:-1]) + 1
    bounds = np.concatenate([[0], change, [flat.size]])
    runs = np.diff(bounds).tolist()
    if flat[0] == 1:
        runs = [0] + runs
    return [int(r) for r in runs]


def _counts_to_string(cnts: Sequence[int]) -> str:
    out = []
    for i, c in enumerate(cnts):
        x = int(c)
        if i > 2:
            x -= int(cnts[i - 2])
        more = True
        while more:
            ch = x & 0x1F
            x >>= 5
            more = (x != -1) if (ch & 0x10) else (x != 0)
            if more:
                ch |= 0x20
            out.append(chr(ch + 48))
    return "".join(out)


def _string_to_counts(s: Union[str, bytes]) -> List[int]:
    if isinstance(s, bytes):
        s = s.decode("ascii")
    cnts: List[int] = []
    p = 0
    while p < len(s):
        x, k, more = 0, 0, True
        while more:
            c = ord(s[p]) - 48
            x |= (c & 0x1F) << (5 * k)
            more = bool(c & 0x20)
            p += 1
            k += 1
            if not more and (c & 0x10):
                x |= -1 << (5 * k)
        if len(cnts) > 2:
            x += cnts[-2]
        cnts.append(x)
    return cnts


def rle_encode(mask: Union[np.ndarray, Tensor]) -> Dict[str, Any]:
    """Encode an ``[H, W]`` binary mask into a compressed COCO RLE ``{"size": [H, W], "counts": str}``."""
    if isinstance(mask, Tensor):
        mask = mask.detach().cpu().numpy()
    h, w = mask.shape
    return {"size": [int(h), int(w)], "counts": _counts_to_string(_runs(mask))}


def _rle_counts(rle: Dict[str, Any]) -> List[int]:
    counts = rle["counts"]
    return list(counts) if isinstance(counts, (list, tuple)) else _string_to_counts(counts)


def rle_decode(rle: Dict[str, Any]) -> np.ndarray:
    """Decode a (compressed or uncompressed) COCO RLE into an ``[H, W]`` uint8 mask."""
    h, w = rle["size"]
    cnts = _rle_counts(rle)
    vals = np.zeros(len(cnts), dtype=np.uint8)
    vals[1::2] = 1
    flat = np.repeat(vals, np.asarray(cnts, dtype=np.int64))
    if flat.size < h * w:
        flat = np.concatenate([flat, np.zeros(h * w - flat.size, np.uint8)])
    return flat[: h * w].reshape((h, w), order="F")


def rle_area(rle: Dict[str, Any]) -> int:
    return int(sum(_rle_counts(rle)[1::2]))


RleState = Tuple[Tuple[int, int], bytes]  # the reference's per-mask state entry: ((H, W), compressed counts)


def encode_mask_batch(masks: Sequence[Tensor]) -> List[Tuple[RleState, ...]]:
    """Per image ``[K_i, H, W]`` masks -> per image tuple of ``((H, W), counts)`` (the reference's segm state,
    ``mean_ap.py:811-816``).  Images sharing (device, H, W) are encoded by ONE ``tmx::rle_encode`` call (the GPU
    kernels when the masks live there; only the strings come back to the host)."""
    out: List[Tuple[RleState, ...]] = [()] * len(masks)
    groups: Dict[Tuple[Any, int, int], List[int]] = {}
    for i, m in enumerate(masks):
        if m.numel() == 0 or m.shape[0] == 0:
            continue
        groups.setdefault((m.device, int(m.shape[-2]), int(m.shape[-1])), []).append(i)
    native = ops.load()
    for (dev, h, w), idx in groups.items():
        if native and (dev.type == "cpu" or ops.use_native(masks[idx[0]])):
            stack = torch.cat([masks[i].reshape(-1, h, w) for i in idx]) if len(idx) > 1 else masks[idx[0]].reshape(-1, h, w)
            chars, off = torch.ops.tmx.rle_encode(stack)
            buf, o = chars.numpy().tobytes(), off.tolist()
            k = 0
            for i in idx:
                n = int(masks[i].shape[0])
                out[i] = tuple(((h, w), buf[o[k + j]:o[k + j + 1]]) for j in range(n))
                k += n
        else:
            for i in idx:
                out[i] = tuple(((h, w), rle_encode(m)["counts"].encode("ascii")) for m in masks[i])
    return out


def rle_state_area(entry: RleState) -> int:
    return rle_area({"size": list(entry[0]), "counts": entry[1]})


def _tiles(d_sizes: Sequence[int], g_sizes: Sequence[int], tile: int = 16) -> np.ndarray:
    """[T, 3] int32 (image, d0, g0) covering every image's [D_i, G_i] IoU block with tile x tile tiles."""
    d = np.asarray(d_sizes, dtype=np.int64)
    g = np.asarray(g_sizes, dtype=np.int64)
    nd, ng = (d + tile - 1) // tile, (g + tile - 1) // tile
    per = nd * ng
    img = np.repeat(np.arange(len(d)), per)
    if img.size == 0:
        return np.zeros((0, 3), dtype=np.int32)
    first = np.repeat(np.cumsum(per) - per, per)
    local = np.arange(img.size) - first
    ngi = ng[img]
    return np.stack([img, (local // ngi) * tile, (local % ngi) * tile], axis=1).astype(np.int32)


def rle_segm_ious(
    det: Sequence[Tuple[RleState, ...]], gt: Sequence[Tuple[RleState, ...]], gt_crowd: Sequence[Tensor], device: torch.device,
    max_bits_bytes: int = 1 << 31,
) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    """Mask IoU blocks of every image from the RLE states (the reference's COCOeval ``computeIoU`` for segm).

    Returns ``(ious, offsets, det_area, gt_area)``: image i's ``[D_i, G_i]`` IoU block (fp64, crowd ground truth
    divides by the detection area) starts at ``offsets[i]`` of the flat ``ious`` (empty when D_i or G_i is 0), and
    the mask areas of every detection / ground truth in image-major order.  Strings are decoded to bit-packed masks
    on ``device`` (``tmx::rle_decode_bits``) for image chunks of at most ``max_bits_bytes``, and every chunk's IoU
    tiles run in ONE ``tmx::mask_iou_tiles`` launch."""
    n_img = len(gt)
    d_sizes = [len(det[i]) if i < len(det) else 0 for i in range(n_img)]
    g_sizes = [len(t) for t in gt]
    blk = [d * g for d, g in zip(d_sizes, g_sizes)]
    offsets = np.concatenate([[0], np.cumsum(blk)[:-1]]).astype(np.int64) if n_img else np.zeros(0, dtype=np.int64)
    total = int(sum(blk))
    ious = torch.zeros(total, dtype=torch.float64, device=device)
    det_first = np.concatenate([[0], np.cumsum(d_sizes)]).astype(np.int64)
    gt_first = np.concatenate([[0], np.cumsum(g_sizes)]).astype(np.int64)
    det_area = torch.zeros(int(det_first[-1]), dtype=torch.float64, device=device)
    gt_area = torch.zeros(int(gt_first[-1]), dtype=torch.float64, device=device)
    crowd_all = [c.reshape(-1).to(torch.bool).cpu() for c in gt_crowd]
    # images grouped by mask size (all of an image's masks share it), then chunked by decoded-bits bytes
    by_size: Dict[Tuple[int, int], List[int]] = {}
    for i in range(n_img):
        e = (det[i][0] if d_sizes[i] else gt[i][0] if g_sizes[i] else None)
        if e is not None:
            sizes = {(int(x[0][0]), int(x[0][1])) for x in (list(det[i]) if d_sizes[i] else []) + list(gt[i])}
            if len(sizes) > 1:
                # one decode size per image: a mismatch would be clamped by the decoder into wrong IoUs / areas
                raise ValueError(
                    f"Image {i}: predicted and ground-truth masks must have the same spatial size, got {sorted(sizes)}"
                )
            by_size.setdefault((int(e[0][0]), int(e[0][1])), []).append(i)
    for (h, w), imgs in by_size.items():
        words = (h * w + 63) // 64
        chunk: List[int] = []
        masks_in_chunk = 0
        for pos, i in enumerate(imgs + [None]):  # type: ignore[list-item]
            if i is not None and (not chunk or (masks_in_chunk + d_sizes[i] + g_sizes[i]) * words * 8 <= max_bits_bytes):
                chunk.append(i)
                masks_in_chunk += d_sizes[i] + g_sizes[i]
                continue
            _iou_chunk(chunk, det, gt, d_sizes, g_sizes, crowd_all, offsets, det_first, gt_first, h, w, device, ious, det_area, gt_area)
            chunk, masks_in_chunk = ([i], d_sizes[i] + g_sizes[i]) if i is not None else ([], 0)
    return ious, torch.as_tensor(offsets, device=device), det_area, gt_area


def _decode(entries: List[RleState], h: int, w: int, device: torch.device) -> Tuple[Tensor, Tensor]:
    lens = np.fromiter((len(e[1]) for e in entries), dtype=np.int64, count=len(entries))
    off = torch.from_numpy(np.concatenate([[0], np.cumsum(lens)]).astype(np.int64))
    raw = b"".join(e[1] for e in entries)
    chars = torch.frombuffer(bytearray(raw), dtype=torch.uint8) if raw else torch.zeros(0, dtype=torch.uint8)
    return torch.ops.tmx.rle_decode_bits(chars.to(device), off.to(device), h, w)


def _iou_chunk(chunk, det, gt, d_sizes, g_sizes, crowd_all, offsets, det_first, gt_first, h, w, device, ious, det_area, gt_area):
    if not chunk:
        return
    d_entries = [e for i in chunk for e in det[i]]
    g_entries = [e for i in chunk for e in gt[i]]
    dbits, darea = _decode(d_entries, h, w, device)
    gbits, garea = _decode(g_entries, h, w, device)
    dsz = [d_sizes[i] for i in chunk]
    gsz = [g_sizes[i] for i in chunk]
    d_rows = torch.as_tensor(np.concatenate([np.arange(det_first[i], det_first[i] + d_sizes[i]) for i in chunk]), device=device)
    g_rows = torch.as_tensor(np.concatenate([np.arange(gt_first[i], gt_first[i] + g_sizes[i]) for i in chunk]), device=device)
    det_area[d_rows] = darea
    gt_area[g_rows] = garea
    tiles = _tiles(dsz, gsz)
    if tiles.shape[0] == 0:
        return
    crowd = torch.cat([crowd_all[i] for i in chunk]) if chunk else torch.zeros(0, dtype=torch.bool)
    det_off = torch.as_tensor(np.concatenate([[0], np.cumsum(dsz)]), dtype=torch.long)
    gt_off = torch.as_tensor(np.concatenate([[0], np.cumsum(gsz)]), dtype=torch.long)
    out_off = torch.as_tensor(offsets[chunk], dtype=torch.long)
    part = torch.ops.tmx.mask_iou_tiles(
        dbits, gbits, darea, garea, crowd.to(device), det_off.to(device), gt_off.to(device), out_off.to(device),
        torch.from_numpy(tiles).to(device), ious.numel(),
    )
    ious.add_(part)


# ------------------------------------------------------------------------------------------------------------
# polygons
# ------------------------------------------------------------------------------------------------------------
def _poly_counts(xy: Sequence[float], h: int, w: int) -> List[int]:
    scale = 5.0
    k = len(xy) // 2
    x = [int(scale * xy[2 * j] + 0.5) for j in range(k)] + [0]
    y = [int(scale * xy[2 * j + 1] + 0.5) for j in range(k)] + [0]
    x[k], y[k] = x[0], y[0]
    u: List[int] = []
    v: List[int] = []
    for j in range(k):
        xs, xe, ys, ye = x[j], x[j + 1], y[j], y[j + 1]
        dx, dy = abs(xe - xs), abs(ys - ye)
        flip = (dx >= dy and xs > xe) or (dx < dy and ys > ye)
        if flip:
            xs, xe, ys, ye = xe, xs, ye, ys
        if dx >= dy:
            s = (ye - ys) / dx if dx else 0.0
            for d in range(dx + 1):
                t = dx - d if flip else d
                u.append(t + xs)
                v.append(int(ys + s * t + 0.5))
        else:
            s = (xe - xs) / dy if dy else 0.0
            for d in range(dy + 1):
                t = dy - d if flip else d
                v.append(t + ys)
                u.append(int(xs + s * t + 0.5))
    px: List[int] = []
    py: List[int] = []
    for j in range(1, len(u)):
        if u[j] == u[j - 1]:
            continue
        xd = float(u[j] if u[j] < u[j - 1] else u[j] - 1)
        xd = (xd + 0.5) / scale - 0.5
        if math.floor(xd) != xd or xd < 0 or xd > w - 1:
            continue
        yd = float(v[j] if v[j] < v[j - 1] else v[j - 1])
        yd = (yd + 0.5) / scale - 0.5
        yd = min(max(yd, 0.0), float(h))
        yd = math.ceil(yd)
        px.append(int(xd))
        py.append(int(yd))
    a = sorted([px[j] * h + py[j] for j in range(len(px))] + [h * w])
    prev = 0
    for j in range(len(a)):
        a[j], prev = a[j] - prev, a[j]
    b: List[int] = []
    j = 0
    b.append(a[j])
    j += 1
    while j < len(a):
        if a[j] > 0:
            b.append(a[j])
            j += 1
        else:
            j += 1
            if j < len(a):
                b[-1] += a[j]
                j += 1
    return b


def poly_to_mask(polys: Sequence[Sequence[float]], h: int, w: int) -> np.ndarray:
    """Rasterise (the union of) COCO polygons into an ``[H, W]`` uint8 mask."""
    out = np.zeros((h, w), dtype=np.uint8)
    for poly in polys:
        out |= rle_decode({"size": [h, w], "counts": _poly_counts(poly, h, w)})
    return out


def segmentation_to_mask(segm: Any, h: int, w: int) -> np.ndarray:
    """COCO ``segmentation`` field (polygons, uncompressed or compressed RLE) -> ``[H, W]`` uint8 mask."""
    if isinstance(segm, list):
        return poly_to_mask(segm, h, w)
    return rle_decode(segm)


# ------------------------------------------------------------------------------------------------------------
# pairwise IoU
# ------------------------------------------------------------------------------------------------------------
def pack_bits(masks: Tensor) -> Tensor:
    """``[N, H, W]`` binary masks -> ``[N, ceil(H*W/64)]`` int64 words (pixel p -> bit p % 64 of word p // 64)."""
    n = masks.shape[0]
    flat = masks.reshape(n, -1).to(torch.bool)
    pad = (-flat.shape[1]) % 64
    if pad:
        flat = torch.nn.functional.pad(flat, (0, pad))
    weights = torch.ones(64, dtype=torch.int64, device=masks.device) << torch.arange(64, device=masks.device)
    return (flat.view(n, -1, 64).to(torch.int64) * weights).sum(-1)


def mask_iou(det: Tensor, gt: Tensor, crowd: Tensor) -> Tensor:
    """Pairwise IoU ``[D, G]`` (fp64) of binary masks ``[D, H, W]`` x ``[G, H, W]`` (crowd: inter / det area)."""
    d_n, g_n = det.shape[0], gt.shape[0]
    if d_n == 0 or g_n == 0:
        return torch.zeros(d_n, g_n, dtype=torch.float64, device=det.device)
    darea = det.reshape(d_n, -1).sum(1).double()
    garea = gt.reshape(g_n, -1).sum(1).double()
    if det.is_cuda and ops.use_native(det):
        return torch.ops.tmx.mask_iou(pack_bits(det), pack_bits(gt.to(det.device)), darea, garea.to(det.device), crowd.to(det.device).bool())
    acc = torch.float32 if det[0].numel() < (1 << 24) else torch.float64
    inter = det.reshape(d_n, -1).to(acc) @ gt.reshape(g_n, -1).to(acc).T
    inter = inter.double()
    union = torch.where(crowd.bool().to(det.device)[None, :], darea[:, None], darea[:, None] + garea[None, :] - inter)
    return torch.where(union > 0, inter / union.clamp_min(1e-300), torch.zeros_like(inter))
