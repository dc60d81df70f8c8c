"""``forward`` vs ``update`` at BASELINE config 2 (VERDICT r3 "make forward cheap and measure it"):
``MetricCollection({MulticlassAUROC, MulticlassConfusionMatrix})``, C = 1000, batch 65536 bf16 logits, 4 pre-generated
batches cycled.  Times K ``update`` calls and K ``coll(preds, target)`` calls (each returns the batch's AUROC and
confusion matrix and accumulates), device-synchronised, after warm-up; prints one JSON line.

    python tools/forward_bench.py [--steps 20] [--warmup 5] [--classes 1000] [--batch 65536]
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
    ap.add_argument("--classes", type=int, default=1000)
    ap.add_argument("--batch", type=int, default=65536)
    args = ap.parse_args()
    import torch

    import torchmetrics_forked_amd as tm
    from torchmetrics_forked_amd import ops

    ops.require()
    dev = torch.device("cuda", 0)
    C, B = args.classes, args.batch
    g = torch.Generator(device=dev).manual_seed(7)
    pool = [(torch.randn(B, C, device=dev, generator=g).bfloat16(), torch.randint(0, C, (B,), device=dev, generator=g)) for _ in range(4)]

    def make():
        return tm.MetricCollection({"auroc": tm.MulticlassAUROC(num_classes=C), "confmat": tm.MulticlassConfusionMatrix(num_classes=C)}).to(dev)

    res = {"config": f"MulticlassAUROC+MulticlassConfusionMatrix C={C} bs={B} bf16", "steps": args.steps}
    for mode in ("update", "forward"):
        coll = make()
        step = coll.update if mode == "update" else coll.__call__
        for i in range(args.warmup):
            step(*pool[i % 4])
        torch.cuda.synchronize(dev)
        best = None
        for rep in range(3):
            torch.cuda.synchronize(dev)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            e0.record()
            for i in range(args.steps):
                out = step(*pool[i % 4])
            e1.record()
            t_enq = time.perf_counter()
            torch.cuda.synchronize(dev)
            dt = (time.perf_counter() - t0) / args.steps
            if best is None or dt < best:
                best = dt
                res[f"{mode}_host_enqueue_us"] = round((t_enq - t0) / args.steps * 1e6, 1)
                res[f"{mode}_gpu_span_us"] = round(e0.elapsed_time(e1) / args.steps * 1e3, 1)
        res[f"{mode}_ms"] = round(best * 1e3, 4)
        # device kernels per step (profiler; GPU time by kernel)
        with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]) as prof:
            for i in range(args.steps):
                out = step(*pool[i % 4])
            torch.cuda.synchronize(dev)
        kern = [(ka.key[:60], round(ka.count / args.steps, 2), round(ka.device_time_total / args.steps, 1))
                for ka in prof.key_averages() if ka.device_time_total > 0 and ka.self_device_time_total > 0]
        res[f"{mode}_device_us_per_step"] = sorted(kern, key=lambda k: -k[2])[:14]
        host = [(ka.key[:60], round(ka.count / args.steps, 2), round(ka.self_cpu_time_total / args.steps, 1))
                for ka in prof.key_averages() if ka.self_cpu_time_total > 0]
        res[f"{mode}_host_us_per_step"] = sorted(host, key=lambda k: -k[2])[:14]
        if mode == "forward":
            res["last_batch_auroc"] = float(out["auroc"])
    res["forward_over_update"] = round(res["forward_ms"] / res["update_ms"], 3)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
