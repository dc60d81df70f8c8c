"""Does the first update after compute() + reset() allocate fresh device segments (hipMalloc) in the headline
collection?  Prints the caching allocator's segment counter and host time around each of the first updates."""
import json
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
g = torch.Generator(device=dev).manual_seed(0)
pool = [(torch.randn(B, C, device=dev, generator=g).bfloat16(), torch.randint(0, C, (B,), device=dev, generator=g)) for _ in range(4)]


def seg():
    s = torch.cuda.memory_stats(dev)
    return s.get("segment.all.allocated", 0), s.get("allocation.all.allocated", 0)


log = []
for phase in ("warmup", "timed"):
    for i in range(5):
        torch.cuda.synchronize()
        s0 = seg()
        t0 = time.perf_counter()
        coll.update(*pool[i % 4])
        host = 1e6 * (time.perf_counter() - t0)
        torch.cuda.synchronize()
        s1 = seg()
        log.append({"phase": phase, "i": i, "host_us": round(host, 1), "new_segments": s1[0] - s0[0], "allocs": s1[1] - s0[1]})
    s0 = seg()
    coll.compute()
    torch.cuda.synchronize()
    log.append({"phase": phase, "compute_new_segments": seg()[0] - s0[0]})
    coll.reset()
    torch.cuda.synchronize()
print(json.dumps(log, indent=0))
