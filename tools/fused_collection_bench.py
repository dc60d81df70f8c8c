"""Update time of MetricCollection {AUROC, ConfusionMatrix} vs {AUROC, ConfusionMatrix, Accuracy, F1} (and a few
more stat members) at 65536 x 1000 bf16: the stat members ride on the fused row pass (ops/fused.py)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import torchmetrics_forked_amd as tm  # noqa: E402


def bench(members, steps=30, n=65536, c=1000, dtype=torch.bfloat16):
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    pool = [(torch.randn(n, c, device=dev, generator=g).to(dtype), torch.randint(0, c, (n,), device=dev, generator=g)) for _ in range(2)]
    coll = tm.MetricCollection(members).to(dev)
    for i in range(5):
        coll.update(*pool[i % 2])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        coll.update(*pool[i % 2])
    torch.cuda.synchronize()
    return 1e3 * (time.perf_counter() - t0) / steps


if __name__ == "__main__":
    C = 1000
    base = lambda: {"auroc": tm.MulticlassAUROC(num_classes=C), "cm": tm.MulticlassConfusionMatrix(num_classes=C)}
    r = {}
    r["auroc+cm"] = bench(base())
    r["auroc+cm+acc+f1"] = bench({**base(), "acc": tm.MulticlassAccuracy(num_classes=C), "f1": tm.MulticlassF1Score(num_classes=C)})
    r["auroc+cm+acc+f1+prec+rec"] = bench({**base(), "acc": tm.MulticlassAccuracy(num_classes=C), "f1": tm.MulticlassF1Score(num_classes=C),
                                           "prec": tm.MulticlassPrecision(num_classes=C), "rec": tm.MulticlassRecall(num_classes=C)})
    r["acc+f1+prec+rec (no curve)"] = bench({"acc": tm.MulticlassAccuracy(num_classes=C), "f1": tm.MulticlassF1Score(num_classes=C),
                                             "prec": tm.MulticlassPrecision(num_classes=C), "rec": tm.MulticlassRecall(num_classes=C)})
    r["acc alone"] = bench({"acc": tm.MulticlassAccuracy(num_classes=C)})
    print(json.dumps({"what": "MetricCollection update ms at 65536 x 1000 bf16 (mean of 30)", "ms_per_update": {k: round(v, 4) for k, v in r.items()},
                      "ratio_with_stats": round(r["auroc+cm+acc+f1"] / r["auroc+cm"], 3)}))
