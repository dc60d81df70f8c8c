"""What does the FIRST timed window of a process (bench.py's only window) do that a repeated window does not?

Headline config (MulticlassAUROC + MulticlassConfusionMatrix, C = 1000, 65536 bf16 rows).  bench.py's sequence --
5 warmup updates + compute + reset + synchronize -- then window A (20 updates + compute, under torch.profiler), the same
cycle again, and window B.  Prints one JSON line: per window the host-op and device-kernel counts / self times, the ops
and kernels that occur in A but not B (or more often), allocator calls (hipMalloc / hipHostMalloc / hipMemset) and the
un-profiled timing of both windows (bench.py's compute_incl_sync = elapsed - GPU update time).

    python tools/window_trace.py [--steps 20]
"""
import argparse
import json
import os
import sys
import time
from collections import Counter, defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()
    import torch

    import torchmetrics_forked_amd as tm
    from torchmetrics_forked_amd import ops

    ops.require()
    dev = torch.device("cuda", 0)
    C, B = 1000, 65536
    g = torch.Generator(device=dev).manual_seed(1234)
    pool = [(torch.randn(B, C, device=dev, generator=g).bfloat16(), torch.randint(0, C, (B,), device=dev, generator=g)) for _ in range(4)]
    coll = tm.MetricCollection({"auroc": tm.MulticlassAUROC(num_classes=C), "confmat": tm.MulticlassConfusionMatrix(num_classes=C)}).to(dev)

    def warm() -> None:
        for i in range(5):
            coll.update(*pool[i % 4])
        coll.compute()
        coll.reset()
        torch.cuda.synchronize(dev)

    def window() -> dict:
        ea, eb = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        ea.record()
        for i in range(args.steps):
            coll.update(*pool[i % 4])
        eb.record()
        t1 = time.perf_counter()
        coll.compute()
        t2 = time.perf_counter()
        torch.cuda.synchronize(dev)
        t3 = time.perf_counter()
        upd = ea.elapsed_time(eb) * 1e3
        return {"incl_sync_us": round((t3 - t0) * 1e6 - upd, 1), "gpu_upd_us_per_step": round(upd / args.steps, 2),
                "enqueue_us": round((t1 - t0) * 1e6, 1), "compute_call_us": round((t2 - t1) * 1e6, 1), "sync_us": round((t3 - t2) * 1e6, 1)}

    out = {"steps": args.steps}
    # un-profiled: first window of the process, then three repeats
    warm()
    out["timing_first"] = window()
    reps = []
    for _ in range(3):
        warm()
        reps.append(window())
    out["timing_repeats"] = reps

    def profiled() -> dict:
        warm()
        with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]) as prof:
            window()
        host, dev_k = Counter(), Counter()
        host_us, dev_us = defaultdict(float), defaultdict(float)
        for e in prof.events():
            name = e.name[:90]
            if e.device_type == torch.autograd.DeviceType.CUDA:
                dev_k[name] += 1
                dev_us[name] += e.device_time_total if hasattr(e, "device_time_total") else 0.0
            else:
                host[name] += 1
                host_us[name] += e.self_cpu_time_total
        return {"host": host, "dev": dev_k, "host_us": host_us, "dev_us": dev_us}

    # a fresh process is not available here: compare a profiled window right after the first warm cycle of a NEW
    # collection (first use of its buffers) with a repeated one
    coll = tm.MetricCollection({"auroc": tm.MulticlassAUROC(num_classes=C), "confmat": tm.MulticlassConfusionMatrix(num_classes=C)}).to(dev)
    a = profiled()
    b = profiled()
    diff_host = {k: [a["host"][k], b["host"].get(k, 0), round(a["host_us"][k], 1)] for k in a["host"] if a["host"][k] > b["host"].get(k, 0)}
    diff_dev = {k: [a["dev"][k], b["dev"].get(k, 0), round(a["dev_us"][k], 1)] for k in a["dev"] if a["dev"][k] > b["dev"].get(k, 0)}
    out["ops_more_in_first"] = dict(sorted(diff_host.items(), key=lambda kv: -kv[1][2])[:40])
    out["kernels_more_in_first"] = diff_dev
    out["host_top_first"] = sorted(((k, a["host"][k], round(v, 1)) for k, v in a["host_us"].items()), key=lambda x: -x[2])[:25]
    out["host_top_repeat"] = sorted(((k, b["host"][k], round(v, 1)) for k, v in b["host_us"].items()), key=lambda x: -x[2])[:25]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
