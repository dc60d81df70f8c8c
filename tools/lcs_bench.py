"""ROUGE-L LCS lengths for 8192 pairs of 512-token documents: host bit-parallel kernel (tmx::lcs_batch, threads over
pairs) vs the GPU wave kernel (tmx::lcs_gpu, incl. H2D of the packed ids and the D2H of the lengths). One JSON line."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from torchmetrics_forked_amd import ops  # noqa: E402

ops.require()
n, L, V = 8192, 512, 2000
g = torch.Generator().manual_seed(0)
a = torch.randint(0, V, (n * L,), generator=g)
b = torch.randint(0, V, (n * L,), generator=g)
off = torch.arange(0, n * L + 1, L)
t0 = time.perf_counter()
host = torch.ops.tmx.lcs_batch(a, off, b, off)
t_host = time.perf_counter() - t0
for _ in range(2):
    torch.ops.tmx.lcs_gpu(a.cuda(), off.cuda(), b.cuda(), off.cuda(), L).cpu()
torch.cuda.synchronize()
t0 = time.perf_counter()
dev = torch.ops.tmx.lcs_gpu(a.cuda(), off.cuda(), b.cuda(), off.cuda(), L).cpu()
t_gpu = time.perf_counter() - t0
assert torch.equal(host, dev)
print(json.dumps({"pairs": n, "tokens": L, "host_ms": round(t_host * 1e3, 1), "gpu_ms_incl_copies": round(t_gpu * 1e3, 2),
                  "speedup": round(t_host / t_gpu, 1)}), flush=True)
