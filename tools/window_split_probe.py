"""Split bench.py's timed window (headline config) into host-timestamped pieces, to find the fixed cost that
``compute_incl_sync_ms`` (elapsed - GPU update time) reports.  Same sequence as bench.py: t0, two timing events,
ev_start.record(), ``--steps`` updates, ev_upd.record(), compute(), synchronize, synchronize.  Runs it with the events
created inside the window (as bench.py did through round 5) and created before t0, and at 20 and 40 steps (the slope is
the true per-update cost, the intercept the window's fixed cost).  Prints one JSON line of medians (us)."""
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
C, B = 1000, 65536
g = torch.Generator(device=dev).manual_seed(1234)
pool = [(torch.randn(B, C, device=dev, generator=g).bfloat16(), torch.randint(0, C, (B,), device=dev, generator=g)) for _ in range(4)]
coll = tm.MetricCollection({"auroc": tm.MulticlassAUROC(num_classes=C), "confmat": tm.MulticlassConfusionMatrix(num_classes=C)}).to(dev)


def window(steps: int, pre_events: bool) -> dict:
    for i in range(5):
        coll.update(*pool[i % 4])
    coll.compute()
    coll.reset()
    torch.cuda.synchronize(dev)
    if pre_events:
        ea, eb = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    if not pre_events:
        ea, eb = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t1 = time.perf_counter()
    ea.record()
    t2 = time.perf_counter()
    for i in range(steps):
        coll.update(*pool[i % 4])
    t3 = time.perf_counter()
    eb.record()
    t4 = time.perf_counter()
    coll.compute()
    t5 = time.perf_counter()
    torch.cuda.synchronize(dev)
    t6 = time.perf_counter()
    torch.cuda.synchronize(dev)
    t7 = time.perf_counter()
    upd = ea.elapsed_time(eb) * 1e3
    us = lambda a, b: (b - a) * 1e6  # noqa: E731
    return {"create_events": us(t0, t1), "record_start": us(t1, t2), "enqueue_updates": us(t2, t3), "record_upd": us(t3, t4),
            "compute_call": us(t4, t5), "sync1": us(t5, t6), "sync2": us(t6, t7), "elapsed": us(t0, t7), "gpu_updates": upd,
            "incl_sync": us(t0, t7) - upd}


out = {}
for steps in (20, 40):
    for pre in (False, True):
        runs = [window(steps, pre) for _ in range(9)]
        key = f"steps{steps}_{'pre' if pre else 'in'}_events"
        out[key] = {k: round(sorted(r[k] for r in runs)[4], 1) for k in runs[0]}
        out[key]["runs_incl_sync"] = [round(r["incl_sync"], 1) for r in runs]
        out[key]["runs_gpu_updates"] = [round(r["gpu_updates"], 1) for r in runs]
        out[key]["runs_compute_call"] = [round(r["compute_call"], 1) for r in runs]
print(json.dumps(out), flush=True)
