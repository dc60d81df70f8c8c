"""Host cost of the headline collection's compute() (BASELINE config 2): wall time with an idle GPU, and a cProfile of
20 computes (each after one update), to find the Python / C++ host work that the driver's short window exposes
(``compute_incl_sync_ms`` of bench.py).  Prints one JSON line, then the profile table."""
import cProfile
import json
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
C, B = 1000, 65536
coll = tm.MetricCollection({"auroc": tm.MulticlassAUROC(num_classes=C), "confmat": tm.MulticlassConfusionMatrix(num_classes=C)}).to(dev)
x = torch.randn(B, C, device=dev).bfloat16()
t = torch.randint(0, C, (B,), device=dev)
for _ in range(3):
    coll.update(x, t)
coll.compute()
walls, hosts = [], []
for _ in range(20):
    coll.update(x, t)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    coll.compute()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    walls.append(1e3 * (time.perf_counter() - t0))
    hosts.append(1e3 * (t1 - t0))
pr = cProfile.Profile()
for _ in range(20):
    coll.update(x, t)
    torch.cuda.synchronize()
    pr.enable()
    coll.compute()
    pr.disable()
torch.cuda.synchronize()
walls.sort()
hosts.sort()
print(json.dumps({"compute_wall_ms_median": walls[len(walls) // 2], "compute_wall_ms_min": walls[0],
                  "compute_host_return_ms_median": hosts[len(hosts) // 2]}), flush=True)
st = pstats.Stats(pr).stats  # {(file, line, fn): (cc, nc, tt, ct, callers)}
rows = sorted(((v[2], v[3], v[1], k) for k, v in st.items()), reverse=True)[:40]
print("tottime_us_per_compute cumtime_us_per_compute ncalls function")
for tt, ct, nc, k in rows:
    print(f"{1e6 * tt / 20:9.1f} {1e6 * ct / 20:9.1f} {nc:6d} {os.path.basename(k[0])}:{k[1]}({k[2]})")
rows = sorted(((v[3], v[2], v[1], k) for k, v in st.items()), reverse=True)[:25]
print("--- by cumulative")
for ct, tt, nc, k in rows:
    print(f"{1e6 * ct / 20:9.1f} {1e6 * tt / 20:9.1f} {nc:6d} {os.path.basename(k[0])}:{k[1]}({k[2]})")
