"""Update throughput of the binary / multilabel exact-histogram curve path (BinaryAUROC, MultilabelAUROC)."""
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
for N in (1 << 20, 1 << 24):
    p = torch.randn(N, device=dev).bfloat16()
    t = torch.randint(0, 2, (N,), device=dev)
    m = tm.BinaryAUROC().to(dev)
    out[f"binary_auroc_update_N{N}_ms"] = round(1e3 * timed(lambda: m.update(p, t)), 3)
for N, L in ((65536, 100), (16384, 1000)):
    p = torch.randn(N, L, device=dev).bfloat16()
    t = torch.randint(0, 2, (N, L), device=dev)
    m = tm.MultilabelAUROC(num_labels=L).to(dev)
    out[f"multilabel_auroc_update_N{N}_L{L}_ms"] = round(1e3 * timed(lambda: m.update(p, t)), 3)
print(out)
