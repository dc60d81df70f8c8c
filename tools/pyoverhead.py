import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import time, torch, torchmetrics_forked_amd as tm
from torchmetrics_forked_amd import ops
ops.require()
dev = torch.device("cuda", 0)
C = 1000
coll = tm.MetricCollection({"auroc": tm.MulticlassAUROC(num_classes=C), "confmat": tm.MulticlassConfusionMatrix(num_classes=C)}).to(dev)
for B in (64, 65536):
    x = torch.randn(B, C, device=dev).bfloat16(); t = torch.randint(0, C, (B,), device=dev)
    for _ in range(5): coll.update(x, t)
    torch.cuda.synchronize()
    n = 200
    t0 = time.perf_counter()
    for _ in range(n): coll.update(x, t)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"B={B}: host enqueue {1e6*(t1-t0)/n:.1f} us/update, wall {1e6*(t2-t0)/n:.1f} us/update")
import cProfile, pstats
x = torch.randn(64, C, device=dev).bfloat16(); t = torch.randint(0, C, (64,), device=dev)
pr = cProfile.Profile(); pr.enable()
for _ in range(500): coll.update(x, t)
pr.disable(); torch.cuda.synchronize()
pstats.Stats(pr).sort_stats("tottime").print_stats(18)
