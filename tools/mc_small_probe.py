"""MulticlassAUROC update cost across class counts (two-pass path needs C % 8 == 0; others take the generic kernel)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import torchmetrics_forked_amd as tm  # noqa: E402
from torchmetrics_forked_amd import ops  # noqa: E402

ops.require()
dev = torch.device("cuda", 0)


def timed(fn, n=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n


out = {}
CONFIGS = ((2, 1 << 20), (10, 1 << 20), (16, 1 << 20), (64, 1 << 20), (100, 1 << 18), (104, 1 << 18), (256, 1 << 18),
           (1000, 1 << 16), (1001, 1 << 16))
if os.environ.get("PROBE_SMALL_ONLY"):
    CONFIGS = CONFIGS[:4]
if os.environ.get("PROBE_CONFIGS"):  # "C:N,C:N,..."
    CONFIGS = tuple(tuple(int(v) for v in cn.split(":")) for cn in os.environ["PROBE_CONFIGS"].split(","))
for C, N in CONFIGS:
    p = torch.randn(N, C, device=dev).bfloat16()
    t = torch.randint(0, C, (N,), device=dev)
    m = tm.MulticlassAUROC(num_classes=C).to(dev)
    ms = 1e3 * timed(lambda: m.update(p, t))
    torch.cuda.synchronize()
    h0 = time.perf_counter()
    for _ in range(10):
        m.update(p, t)
    host_us = 1e5 * (time.perf_counter() - h0)  # enqueue only (no synchronisation): the host cost per update
    torch.cuda.synchronize()
    out[f"C{C}_N{N}"] = {"ms": round(ms, 4), "host_us": round(host_us, 1), "input_TBps": round(p.numel() * 2 / (ms * 1e-3) / 1e12, 3)}
print(json.dumps(out))
