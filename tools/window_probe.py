"""Where the headline's timed window goes (VERDICT r3 "attribute every us between t0 and the end"): the exact bench.py
window (``--warmup`` updates + compute + reset, then ``--steps`` updates + ONE compute) under torch.profiler, reporting

* host time to enqueue the updates, host time inside ``compute()`` and where it blocked (runtime calls > 20 us:
  synchronising copies / stream syncs), and the GPU time of the compute's kernels;
* the same window without the profiler (plain perf_counter + events), for reference.

    python tools/window_probe.py [--steps 20] [--warmup 5]

Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
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

    def window(profile: bool) -> dict:
        for i in range(args.warmup):
            coll.update(*pool[i % 4])
        coll.compute()
        coll.reset()
        torch.cuda.synchronize(dev)
        out = {}
        ctx = torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]) if profile else None
        if ctx:
            ctx.__enter__()
        t0 = time.perf_counter()
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        e0.record()
        for i in range(args.steps):
            coll.update(*pool[i % 4])
        t_enq = time.perf_counter()
        e1.record()
        coll.compute()
        t_cmp = time.perf_counter()
        e2.record()
        torch.cuda.synchronize(dev)
        t_end = time.perf_counter()
        if ctx:
            ctx.__exit__(None, None, None)
        out.update(
            host_enqueue_updates_ms=round((t_enq - t0) * 1e3, 3), host_compute_call_ms=round((t_cmp - t_enq) * 1e3, 3),
            wall_ms=round((t_end - t0) * 1e3, 3), gpu_updates_ms=round(e0.elapsed_time(e1), 3), gpu_compute_ms=round(e1.elapsed_time(e2), 3),
        )
        if ctx:
            blocking = []
            kernels = []
            for ev in ctx.events():
                name = ev.name
                dur = ev.cpu_time_total if hasattr(ev, "cpu_time_total") else 0
                if any(k in name for k in ("Memcpy", "Synchronize", "memcpy", "synchronize", "EventSynchronize", "StreamSynchronize")) and dur > 20:
                    blocking.append((name, round(dur, 1)))
            for ka in ctx.key_averages():
                if ka.device_time_total > 0 and ka.count <= 64:
                    kernels.append((ka.key[:80], ka.count, round(ka.device_time_total, 1)))
            out["blocking_runtime_calls_us"] = blocking[:20]
            out["device_ops_us"] = sorted(kernels, key=lambda k: -k[2])[:25]
        return out

    res = {"plain": [window(False) for _ in range(3)], "profiled": window(True)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
