"""torch.profiler breakdown of the headline collection's compute() (MulticlassAUROC + ConfusionMatrix, C=1000)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import torchmetrics_forked_amd as tm  # noqa: E402
from torchmetrics_forked_amd import ops  # noqa: E402

ops.require()
dev = torch.device("cuda", 0)
C, N = 1000, 65536
g = torch.Generator(device=dev).manual_seed(0)
x = torch.randn(N, C, device=dev, generator=g).bfloat16()
t = torch.randint(0, C, (N,), device=dev, generator=g)
coll = tm.MetricCollection({"auroc": tm.MulticlassAUROC(num_classes=C), "cm": tm.MulticlassConfusionMatrix(num_classes=C)}).to(dev)
for _ in range(5):
    coll.update(x, t)
coll.compute()
torch.cuda.synchronize()
import time  # noqa: E402

t0 = time.perf_counter()
for _ in range(5):
    coll._computed = None
    for m in coll.values(copy_state=False):
        m._computed = None
    coll.compute()
torch.cuda.synchronize()
print(f"compute: {(time.perf_counter() - t0) / 5 * 1e3:.3f} ms")
with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]) as prof:
    for m in coll.values(copy_state=False):
        m._computed = None
    coll.compute()
    torch.cuda.synchronize()
print(prof.key_averages().table(sort_by="self_cuda_time_total", row_limit=15, max_name_column_width=60))
print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=15, max_name_column_width=60))
