"""Where the end-of-window compute() of the headline collection spends its time (host vs kernels)."""
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
coll = tm.MetricCollection({"auroc": tm.MulticlassAUROC(num_classes=C), "confmat": tm.MulticlassConfusionMatrix(num_classes=C)}).to(dev)
x = torch.randn(B, C, device=dev).bfloat16()
t = torch.randint(0, C, (B,), device=dev)
for _ in range(3):
    coll.update(x, t)
coll.compute()
times = []
for _ in range(5):
    coll.update(x, t)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    coll.compute()
    torch.cuda.synchronize()
    times.append(1e3 * (time.perf_counter() - t0))
print("compute ms:", [round(v, 3) for v in times])
coll.update(x, t)
torch.cuda.synchronize()
with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]) as prof:
    coll.compute()
    torch.cuda.synchronize()
print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=25))
