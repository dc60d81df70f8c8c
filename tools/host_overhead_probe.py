"""Host cost of one ``update`` (VERDICT r3 "cut per-update host cost on the GPU"): small device batches, so the
GPU is never the bottleneck; ``host_us`` = wall time of K back-to-back updates / K without synchronising (the
host's enqueue rate), ``wall_us`` = the same with a final synchronize.  Also a cProfile of MulticlassAUROC(C=10)
updates (top functions by own time) to show where the host time goes.

    python tools/host_overhead_probe.py [--k 2000]

Prints one JSON line.
"""
import argparse
import cProfile
import io
import json
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=2000)
    args = ap.parse_args()
    import torch

    import torchmetrics_forked_amd as tm
    from torchmetrics_forked_amd import ops

    ops.require()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)

    def mc(C, n=4096):
        return torch.randn(n, C, device=dev, generator=g).bfloat16(), torch.randint(0, C, (n,), device=dev, generator=g)

    cases = {
        "MulticlassAUROC_C10": (lambda: tm.MulticlassAUROC(num_classes=10), mc(10)),
        "MulticlassAUROC_C1000": (lambda: tm.MulticlassAUROC(num_classes=1000), mc(1000, 256)),
        "MulticlassAccuracy_C10": (lambda: tm.MulticlassAccuracy(num_classes=10), mc(10)),
        "MulticlassConfusionMatrix_C10": (lambda: tm.MulticlassConfusionMatrix(num_classes=10), mc(10)),
        "BinaryAUROC": (lambda: tm.BinaryAUROC(), (torch.rand(4096, device=dev).bfloat16(), torch.randint(0, 2, (4096,), device=dev))),
        "MeanSquaredError": (lambda: tm.MeanSquaredError(), (torch.randn(4096, device=dev), torch.randn(4096, device=dev))),
        "Collection_AUROC_ConfMat_C1000": (
            lambda: tm.MetricCollection({"auroc": tm.MulticlassAUROC(num_classes=1000), "confmat": tm.MulticlassConfusionMatrix(num_classes=1000)}),
            mc(1000, 256),
        ),
    }
    out = {}
    for name, (make, batch) in cases.items():
        m = make().to(dev)
        for _ in range(20):
            m.update(*batch)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(args.k):
            m.update(*batch)
        t1 = time.perf_counter()
        torch.cuda.synchronize(dev)
        t2 = time.perf_counter()
        out[name] = {"host_us": round((t1 - t0) / args.k * 1e6, 2), "wall_us": round((t2 - t0) / args.k * 1e6, 2)}
    m = cases["MulticlassAUROC_C10"][0]().to(dev)
    batch = cases["MulticlassAUROC_C10"][1]
    for _ in range(20):
        m.update(*batch)
    torch.cuda.synchronize(dev)
    prof = cProfile.Profile()
    prof.enable()
    for _ in range(500):
        m.update(*batch)
    prof.disable()
    torch.cuda.synchronize(dev)
    s = io.StringIO()
    pstats.Stats(prof, stream=s).sort_stats("tottime").print_stats(18)
    out["profile_MulticlassAUROC_C10"] = [ln for ln in s.getvalue().splitlines() if ln.strip()][:30]
    # Python time of the headline collection's update (cProfile, own time per function)
    coll = cases["Collection_AUROC_ConfMat_C1000"][0]().to(dev)
    batch = cases["Collection_AUROC_ConfMat_C1000"][1]
    for _ in range(20):
        coll.update(*batch)
    torch.cuda.synchronize(dev)
    prof = cProfile.Profile()
    prof.enable()
    for _ in range(500):
        coll.update(*batch)
    prof.disable()
    torch.cuda.synchronize(dev)
    s = io.StringIO()
    pstats.Stats(prof, stream=s).sort_stats("tottime").print_stats(25)
    out["profile_Collection_C1000"] = [ln for ln in s.getvalue().splitlines() if ln.strip()][:36]
    # Python time of the headline collection's compute() (cProfile over 30 computes, 4 updates before each)
    prof = cProfile.Profile()
    for _ in range(30):
        for _ in range(4):
            coll.update(*batch)
        torch.cuda.synchronize(dev)
        prof.enable()
        coll.compute()
        prof.disable()
        coll.reset()
    s = io.StringIO()
    pstats.Stats(prof, stream=s).sort_stats("tottime").print_stats(30)
    out["profile_Collection_compute"] = [ln for ln in s.getvalue().splitlines() if ln.strip()][:40]
    # host time per update by op / runtime call (torch.profiler, CPU self time): the headline collection
    coll = cases["Collection_AUROC_ConfMat_C1000"][0]().to(dev)
    batch = cases["Collection_AUROC_ConfMat_C1000"][1]
    for _ in range(20):
        coll.update(*batch)
    torch.cuda.synchronize(dev)
    K = 200
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]) as prof2:
        for _ in range(K):
            coll.update(*batch)
        torch.cuda.synchronize(dev)
    rows = []
    for ka in prof2.key_averages():
        if ka.self_cpu_time_total > 0:
            rows.append((ka.key[:70], round(ka.count / K, 2), round(ka.self_cpu_time_total / K, 2)))
    out["collection_host_us_per_update_by_op"] = sorted(rows, key=lambda r: -r[2])[:20]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
