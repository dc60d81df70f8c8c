"""Where does the short headline window lose time?  Replays bench.py's sequence (W warm-up updates, compute, reset,
sync) and then times K updates with a CUDA event after every update and the host clock around every call, printing
per-update GPU time (event to event) and host enqueue time.  A slow first update after reset() or slow early updates
(clock ramp from idle) show up as the first rows."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import torchmetrics_forked_amd as tm  # noqa: E402
from torchmetrics_forked_amd import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--warmup", type=int, default=5)
ap.add_argument("--repeats", type=int, default=3)
args = ap.parse_args()
ops.require()
dev = torch.device("cuda", 0)
C, B = 1000, 65536
coll = tm.MetricCollection({"auroc": tm.MulticlassAUROC(num_classes=C), "confmat": tm.MulticlassConfusionMatrix(num_classes=C)}).to(dev)
gen = torch.Generator(device=dev).manual_seed(1234)
pool = [(torch.randn(B, C, device=dev, generator=gen).bfloat16(), torch.randint(0, C, (B,), device=dev, generator=gen)) for _ in range(4)]
out = []
for rep in range(args.repeats):
    for i in range(args.warmup):
        coll.update(*pool[i % 4])
    coll.compute()
    coll.reset()
    torch.cuda.synchronize()
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 2)]
    host = []
    t0 = time.perf_counter()
    evs[0].record()
    for i in range(args.steps):
        h0 = time.perf_counter()
        coll.update(*pool[i % 4])
        host.append(1e6 * (time.perf_counter() - h0))
        evs[i + 1].record()
    coll.compute()
    evs[-1].record()
    torch.cuda.synchronize()
    wall = 1e3 * (time.perf_counter() - t0)
    gpu = [1e3 * evs[i].elapsed_time(evs[i + 1]) for i in range(args.steps)]
    out.append({"rep": rep, "wall_ms": round(wall, 3), "gpu_us_per_update": [round(x, 1) for x in gpu],
                "host_us_per_update": [round(x, 1) for x in host],
                "compute_us": round(1e3 * evs[-2].elapsed_time(evs[-1]), 1)})
print(json.dumps(out, indent=1))

if os.environ.get("TMX_PROBE_PROFILE"):
    # host-side op breakdown of the first update after the first reset (fresh collection) vs a steady-state update
    coll2 = tm.MetricCollection({"auroc": tm.MulticlassAUROC(num_classes=C), "confmat": tm.MulticlassConfusionMatrix(num_classes=C)}).to(dev)
    for i in range(args.warmup):
        coll2.update(*pool[i % 4])
    coll2.compute()
    coll2.reset()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile

    with profile(activities=[ProfilerActivity.CPU], with_stack=True) as prof:
        coll2.update(*pool[0])
    print("=== first update after reset ===")
    print(prof.key_averages().table(sort_by="cpu_time_total", row_limit=25))
    print("=== first update after reset: stacks of copies / aranges / fills ===")
    for ev in prof.key_averages(group_by_stack_n=12):
        if ev.key in ("aten::copy_", "aten::arange", "aten::cat", "aten::fill_", "aten::zero_", "aten::empty", "aten::add"):
            print(ev.key, round(ev.cpu_time_total, 1), "us")
            for fr in ev.stack:
                if "torchmetrics_forked_amd" in fr:
                    print("    ", fr)
    with profile(activities=[ProfilerActivity.CPU]) as prof:
        coll2.update(*pool[1])
    print("=== steady update ===")
    print(prof.key_averages().table(sort_by="cpu_time_total", row_limit=15))
    import cProfile
    import pstats

    coll2.compute()
    coll2.reset()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    coll2.update(*pool[0])
    pr.disable()
    pstats.Stats(pr).sort_stats("cumulative").print_stats(30)

if os.environ.get("TMX_PROBE_COMPUTE"):
    # host-side op breakdown of the collection compute() that closes the timed window
    coll3 = tm.MetricCollection({"auroc": tm.MulticlassAUROC(num_classes=C), "confmat": tm.MulticlassConfusionMatrix(num_classes=C)}).to(dev)
    for i in range(6):
        coll3.update(*pool[i % 4])
    coll3.compute()
    coll3.reset()
    for i in range(6):
        coll3.update(*pool[i % 4])
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile

    with profile(activities=[ProfilerActivity.CPU], with_stack=True) as prof:
        coll3.compute()
        torch.cuda.synchronize()
    print("=== compute ===")
    print(prof.key_averages().table(sort_by="cpu_time_total", row_limit=30))
    for ev in prof.key_averages(group_by_stack_n=10):
        if ev.key in ("aten::copy_", "aten::to", "aten::cat", "aten::fill_", "aten::zero_", "aten::item", "aten::_local_scalar_dense",
                      "aten::stack", "aten::clone", "aten::div", "aten::mean"):
            print(ev.key, round(ev.cpu_time_total, 1), "us", ev.count)
            for fr in ev.stack[:6]:
                if "torchmetrics_forked_amd" in fr:
                    print("    ", fr)
