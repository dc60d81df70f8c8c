"""fp32 vs bf16 MulticlassAUROC / AveragePrecision at 65536 x 1000: K updates + one compute, per dtype.

bf16 takes the exact-histogram path, fp32 the sample lists + positive-anchored compute (csrc/curve_anchor.hip).
Prints one JSON line per (metric, dtype, K)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import torchmetrics_forked_amd as tm  # noqa: E402


def run(cls, dtype, K, n=65536, c=1000, reps=3):
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    logits = [torch.randn(n, c, device=dev, generator=g).to(dtype) for _ in range(2)]
    target = [torch.randint(0, c, (n,), device=dev, generator=g) for _ in range(2)]
    m = cls(num_classes=c).to(dev)
    best = None
    for r in range(reps + 1):
        m.reset()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(K):
            m.update(logits[i % 2], target[i % 2])
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        v = m.compute()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        if r == 0:
            continue
        cur = (t1 - t0, t2 - t1)
        best = cur if best is None or sum(cur) < sum(best) else best
    return {"metric": cls.__name__, "dtype": str(dtype), "K": K, "update_ms": round(1e3 * best[0] / K, 4),
            "compute_ms": round(1e3 * best[1], 3), "total_ms": round(1e3 * sum(best), 3), "value": float(v)}


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "fp32":  # profiling run: fp32 AUROC only
        print(json.dumps(run(tm.MulticlassAUROC, torch.float32, 10, reps=1)), flush=True)
        sys.exit(0)
    for K in (1, 10):
        for cls in (tm.MulticlassAUROC, tm.MulticlassAveragePrecision):
            for dt in (torch.bfloat16, torch.float32):
                print(json.dumps(run(cls, dt, K)), flush=True)
