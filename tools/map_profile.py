"""Where does BASELINE config 3 (MeanAveragePrecision COCO-80, 512 images x 100 detections / step) spend its time?
The rocprof kernel statistics (profiles/map_kernel_stats_r5.csv) account for ~4 ms of GPU time over 6 updates + 2
computes, against ~4 ms per update and ~19-27 ms per compute of wall time: the config is host-bound.  This probe times
update and compute and prints cProfile tables (per call, us) for both, so the host hot spots are named.

    python tools/map_profile.py        -> one JSON line, then the tables
"""
import cProfile
import json
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from torchmetrics_forked_amd.detection import MeanAveragePrecision  # noqa: E402

dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
n_img, n_det, n_gt, n_cls = 512, 100, 20, 80
g = torch.Generator(device=dev).manual_seed(7)


def batch():
    xy = torch.rand(n_img, n_gt, 2, device=dev, generator=g) * 500
    gt = torch.cat([xy, xy + torch.rand(n_img, n_gt, 2, device=dev, generator=g) * 150 + 4], -1)
    jitter = gt + torch.randn(n_img, n_gt, 4, device=dev, generator=g) * 6
    extra_idx = torch.randint(0, n_gt, (n_img, n_det - n_gt), device=dev, generator=g)
    extra = torch.gather(torch.cat([xy, xy + 50], -1), 1, extra_idx[..., None].expand(-1, -1, 4)) + 30
    det = torch.cat([jitter, extra], 1)
    det[..., 2:] = torch.maximum(det[..., 2:], det[..., :2] + 1)
    gl = torch.randint(0, n_cls, (n_img, n_gt), device=dev, generator=g)
    dl = torch.cat([gl, torch.randint(0, n_cls, (n_img, n_det - n_gt), device=dev, generator=g)], 1)
    sc = torch.rand(n_img, n_det, device=dev, generator=g)
    return [{"boxes": det[i], "scores": sc[i], "labels": dl[i]} for i in range(n_img)], [{"boxes": gt[i], "labels": gl[i]} for i in range(n_img)]


def sync() -> None:
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


pool = [batch() for _ in range(2)]
m = MeanAveragePrecision().to(dev)
m.update(*pool[0])
m.compute()
m.reset()
sync()
steps = 5
t0 = time.perf_counter()
for i in range(steps):
    m.update(*pool[i % 2])
sync()
t1 = time.perf_counter()
res = m.compute()
sync()
t2 = time.perf_counter()
m.reset()
pu, pc = cProfile.Profile(), cProfile.Profile()
pu.enable()
for i in range(steps):
    m.update(*pool[i % 2])
sync()
pu.disable()
pc.enable()
m.compute()
sync()
pc.disable()
print(json.dumps({"device": str(dev), "update_ms": round(1e3 * (t1 - t0) / steps, 3), "compute_ms": round(1e3 * (t2 - t1), 3),
                  "map": round(float(res["map"]), 5)}), flush=True)
for name, pr, calls in (("update", pu, steps), ("compute", pc, 1)):
    st = pstats.Stats(pr).stats
    print(f"--- {name}: by cumulative (us per {name})")
    for ct, tt, nc, k in sorted(((v[3], v[2], v[1], k) for k, v in st.items()), reverse=True)[:30]:
        print(f"{1e6 * ct / calls:10.1f} {1e6 * tt / calls:10.1f} {nc:8d} {os.path.basename(k[0])}:{k[1]}({k[2]})")
    print(f"--- {name}: by self time")
    for tt, ct, nc, k in sorted(((v[2], v[3], v[1], k) for k, v in st.items()), reverse=True)[:25]:
        print(f"{1e6 * tt / calls:10.1f} {1e6 * ct / calls:10.1f} {nc:8d} {os.path.basename(k[0])}:{k[1]}({k[2]})")
