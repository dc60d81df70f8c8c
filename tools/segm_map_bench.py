"""Segmentation mAP at scale on the device: 512 images x (100 detections + 20 ground truths) at 512 x 512, updates of
16 images (masks encoded to COCO RLE by csrc/rle.hip), then compute (one decode + one tiled IoU launch per chunk).
``--check`` also moves the RLE states to the CPU and runs the host evaluator: every output must be identical."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from torchmetrics_forked_amd import ops  # noqa: E402
from torchmetrics_forked_amd.detection import MeanAveragePrecision  # noqa: E402


def box_masks(k, h, w, g, dev):
    x0 = torch.randint(0, w - 8, (k, 1, 1), generator=g, device=dev)
    y0 = torch.randint(0, h - 8, (k, 1, 1), generator=g, device=dev)
    x1 = torch.minimum(x0 + torch.randint(8, w // 2, (k, 1, 1), generator=g, device=dev), torch.tensor(w, device=dev))
    y1 = torch.minimum(y0 + torch.randint(8, h // 2, (k, 1, 1), generator=g, device=dev), torch.tensor(h, device=dev))
    yy = torch.arange(h, device=dev).view(1, h, 1)
    xx = torch.arange(w, device=dev).view(1, 1, w)
    return (yy >= y0) & (yy < y1) & (xx >= x0) & (xx < x1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--images", type=int, default=512)
    ap.add_argument("--per-update", type=int, default=16)
    ap.add_argument("--dets", type=int, default=100)
    ap.add_argument("--gts", type=int, default=20)
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--check", action="store_true")
    args = ap.parse_args()
    ops.require()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    h = w = args.size
    batches = []
    for _ in range(args.images // args.per_update):
        preds, target = [], []
        for _ in range(args.per_update):
            gm = box_masks(args.gts, h, w, g, dev)
            dm = torch.cat([gm, box_masks(args.dets - args.gts, h, w, g, dev)])
            preds.append({"masks": dm, "scores": torch.rand(args.dets, generator=g, device=dev),
                          "labels": torch.randint(0, 10, (args.dets,), generator=g, device=dev)})
            target.append({"masks": gm, "labels": torch.randint(0, 10, (args.gts,), generator=g, device=dev)})
        batches.append((preds, target))
    m = MeanAveragePrecision(iou_type="segm").to(dev)
    m.update(*batches[0])  # warm-up (kernels, allocator)
    m.reset()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for b in batches:
        m.update(*b)
    torch.cuda.synchronize()
    t_upd = time.perf_counter() - t0
    t0 = time.perf_counter()
    res = m.compute()
    torch.cuda.synchronize()
    t_cmp = time.perf_counter() - t0
    chars = sum(len(e[1]) for img in m.detection_mask + m.groundtruth_mask for e in img)
    out = {
        "images": args.images, "masks": args.images * (args.dets + args.gts), "size": [h, w],
        "update_ms_per_image": round(1e3 * t_upd / args.images, 4),
        "mask_pixels_per_s": round(args.images * (args.dets + args.gts) * h * w / t_upd / 1e9, 2),
        "compute_s": round(t_cmp, 4), "rle_state_MB": round(chars / 1e6, 2),
        "dense_bool_state_MB": round(args.images * (args.dets + args.gts) * h * w / 1e6, 1),
        "map": float(res["map"]),
    }
    if args.check:
        cpu = MeanAveragePrecision(iou_type="segm")
        for name in ("detection_mask", "groundtruth_mask"):
            setattr(cpu, name, list(getattr(m, name)))
        for name in ("detection_scores", "detection_labels", "groundtruth_labels", "groundtruth_crowds", "groundtruth_area"):
            setattr(cpu, name, [t.cpu() for t in getattr(m, name)])
        cpu._update_count = 1
        t0 = time.perf_counter()
        ref = cpu.compute()
        out["host_compute_s"] = round(time.perf_counter() - t0, 3)
        out["identical_to_host"] = all(torch.equal(res[k].cpu(), ref[k]) for k in ref)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
