"""Host enqueue time vs wall time per update for common metrics (tiny and large batches)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import torchmetrics_forked_amd as tm  # noqa: E402
from torchmetrics_forked_amd import ops  # noqa: E402

ops.require()
dev = torch.device("cuda", 0)
cases = {
    "MulticlassAccuracy": lambda C: tm.MulticlassAccuracy(num_classes=C),
    "MulticlassF1": lambda C: tm.MulticlassF1Score(num_classes=C),
    "MulticlassConfusionMatrix": lambda C: tm.MulticlassConfusionMatrix(num_classes=C),
}
for name, mk in cases.items():
    for B in (64, 65536):
        C = 1000
        x = torch.randn(B, C, device=dev).bfloat16()
        t = torch.randint(0, C, (B,), device=dev)
        m = mk(C).to(dev)
        for _ in range(5):
            m.update(x, t)
        torch.cuda.synchronize()
        n = 100
        t0 = time.perf_counter()
        for _ in range(n):
            m.update(x, t)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"{name} B={B}: host {1e6 * (t1 - t0) / n:.1f} us, wall {1e6 * (t2 - t0) / n:.1f} us")
m = tm.MulticlassAccuracy(num_classes=1000).to(dev)
x = torch.randn(64, 1000, device=dev).bfloat16()
t = torch.randint(0, 1000, (64,), device=dev)
with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU]) as prof:
    for _ in range(50):
        m.update(x, t)
print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=15))
