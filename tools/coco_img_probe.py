"""Timing probe of the per-image COCO route (tmx::coco_evaluate_gpu_img) on BASELINE config 3's shape: 2560 images x
100 detections + 20 ground truths, 80 classes.  TMX_COCO_IMG_PROBE skips parts of coco_image_match_kernel (bit 0:
ground-truth counts, bit 1: rank pass, bit 2: matching) so each part's cost shows; one JSON line of median us."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from torchmetrics_forked_amd import ops  # noqa: E402
from torchmetrics_forked_amd.detection.mean_ap import _AREA_RANGES  # noqa: E402

ops.require()
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(3)
I, D, G, K = 2560, 100, 20, 80
xy = torch.rand(I, G, 2, device=dev, generator=g) * 500
wh = torch.rand(I, G, 2, device=dev, generator=g) * 150 + 4
gt = torch.cat([xy, wh], -1)
det = torch.cat([gt + torch.randn(I, G, 4, device=dev, generator=g) * 6,
                 torch.cat([torch.rand(I, D - G, 2, device=dev, generator=g) * 500,
                            torch.rand(I, D - G, 2, device=dev, generator=g) * 150 + 4], -1)], 1).abs() + 1
args = (det.reshape(-1, 4).double(), torch.rand(I * D, device=dev, generator=g), torch.randint(0, K, (I * D,), device=dev, generator=g),
        torch.arange(0, I * D + 1, D, device=dev),
        gt.reshape(-1, 4).double(), torch.randint(0, K, (I * G,), device=dev, generator=g), torch.zeros(I * G, dtype=torch.long, device=dev),
        (gt[..., 2] * gt[..., 3]).reshape(-1).double(), torch.arange(0, I * G + 1, G, device=dev), K,
        torch.linspace(0.5, 0.95, 10, dtype=torch.float64, device=dev), torch.linspace(0, 1, 101, dtype=torch.float64, device=dev),
        torch.tensor([1, 10, 100]), torch.tensor([1, 10, 100], device=dev), torch.tensor(_AREA_RANGES, dtype=torch.float64, device=dev))


def med_us(reps=15):
    for _ in range(3):
        torch.ops.tmx.coco_evaluate_gpu_img(*args)
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        torch.ops.tmx.coco_evaluate_gpu_img(*args)
        b.record()
        b.synchronize()
        ts.append(1e3 * a.elapsed_time(b))
    return round(sorted(ts)[len(ts) // 2], 1)


out = {}
for probe in (0, 1, 2, 4, 7):
    os.environ["TMX_COCO_IMG_PROBE"] = str(probe)
    out[f"probe{probe}"] = med_us()
print(json.dumps(out), flush=True)
