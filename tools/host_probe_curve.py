"""Host (enqueue) time per update of the headline collection, with the class pass on the side stream or not, and a
cProfile breakdown of the Python side.  Small batches keep the GPU far ahead of the host."""
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import torchmetrics_forked_amd as tm  # noqa: E402
from torchmetrics_forked_amd import ops  # noqa: E402

ops.require()
dev = torch.device("cuda", 0)
C = 1000
for side in ("1", "0"):
    os.environ["TMX_CURVE_SIDE_STREAM"] = side
    for B in (256, 65536):
        x = torch.randn(B, C, device=dev).bfloat16()
        t = torch.randint(0, C, (B,), device=dev)
        coll = tm.MetricCollection({"auroc": tm.MulticlassAUROC(num_classes=C), "cm": tm.MulticlassConfusionMatrix(num_classes=C)}).to(dev)
        for _ in range(5):
            coll.update(x, t)
        torch.cuda.synchronize()
        n = 100
        t0 = time.perf_counter()
        for _ in range(n):
            coll.update(x, t)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"side={side} B={B}: host {1e6 * (t1 - t0) / n:.1f} us/update, wall {1e6 * (t2 - t0) / n:.1f} us/update", flush=True)
os.environ["TMX_CURVE_SIDE_STREAM"] = "1"
x = torch.randn(256, C, device=dev).bfloat16()
t = torch.randint(0, C, (256,), device=dev)
coll = tm.MetricCollection({"auroc": tm.MulticlassAUROC(num_classes=C), "cm": tm.MulticlassConfusionMatrix(num_classes=C)}).to(dev)
for _ in range(5):
    coll.update(x, t)
pr = cProfile.Profile()
pr.enable()
for _ in range(200):
    coll.update(x, t)
pr.disable()
torch.cuda.synchronize()
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(30)
print(s.getvalue())
