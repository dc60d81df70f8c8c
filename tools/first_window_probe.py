"""Why is the FIRST timed window of a process slower than later ones (headline config; window_split_probe.py: first
window 134 us of fixed cost and 97.6 us per update, later windows ~60 us and ~92 us)?  One variant per process:

* ``base``    -- bench.py's sequence: 5 warmup updates + compute + reset, window 1, then the same again for window 2;
* ``spin``    -- base plus ~300 ms of GPU matmuls before window 1 (is it the clock ramp after an idle GPU?);
* ``double``  -- the warmup cycle (5 updates + compute + reset) twice before window 1 (a second cycle's memory);
* ``inplace`` -- base with reset() zeroing the tensor states in place (the timed window reuses warmed memory);
* ``gccollect`` -- base with gc.collect() before each window; ``gcoff`` -- base with the garbage collector disabled.

    python tools/first_window_probe.py <variant>      -> one JSON line
"""
import gc
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import torchmetrics_forked_amd as tm  # noqa: E402
from torchmetrics_forked_amd import ops  # noqa: E402

variant = sys.argv[1] if len(sys.argv) > 1 else "base"
ops.require()
dev = torch.device("cuda", 0)
C, B = 1000, 65536
g = torch.Generator(device=dev).manual_seed(1234)
pool = [(torch.randn(B, C, device=dev, generator=g, dtype=torch.float32).to(torch.bfloat16), torch.randint(0, C, (B,), device=dev, generator=g))
        for _ in range(4)]
coll = tm.MetricCollection({"auroc": tm.MulticlassAUROC(num_classes=C), "confmat": tm.MulticlassConfusionMatrix(num_classes=C)}).to(dev)

if variant == "inplace":
    for m in coll.values():
        orig = m.reset

        def reset(m=m, orig=orig):  # noqa: ANN001, ANN202
            keep = {n: getattr(m, n) for n, d in m._defaults.items() if isinstance(d, torch.Tensor)}
            orig()
            for n, t in keep.items():
                t.copy_(getattr(m, n))
                setattr(m, n, t)

        m.reset = reset


def warm_cycle() -> None:
    for i in range(5):
        coll.update(*pool[i % 4])
    coll.compute()
    coll.reset()
    torch.cuda.synchronize(dev)


def window(steps: int = 20) -> dict:
    if variant == "gccollect":
        gc.collect()
    ea, eb = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ea.record()
    for i in range(steps):
        coll.update(*pool[i % 4])
    eb.record()
    t1 = time.perf_counter()
    coll.compute()
    t2 = time.perf_counter()
    torch.cuda.synchronize(dev)
    torch.cuda.synchronize(dev)
    t3 = time.perf_counter()
    el = (t3 - t0) * 1e6
    upd = ea.elapsed_time(eb) * 1e3
    return {"upd_us_per_step": round(upd / steps, 2), "incl_sync_us": round(el - upd, 1), "updates_per_s": round(steps / el * 1e6, 1),
            "enqueue_us": round((t1 - t0) * 1e6, 1), "compute_call_us": round((t2 - t1) * 1e6, 1), "syncs_us": round((t3 - t2) * 1e6, 1)}


if variant == "gcoff":
    gc.disable()
warm_cycle()
if variant == "double":
    warm_cycle()
if variant == "spin":
    a = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
    t = time.perf_counter()
    while time.perf_counter() - t < 0.3:
        for _ in range(10):
            a @ a
        torch.cuda.synchronize(dev)
    del a
w1 = window()
warm_cycle()
w2 = window()
print(json.dumps({"variant": variant, "window1": w1, "window2": w2}), flush=True)
