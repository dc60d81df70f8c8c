"""Per-step compute of a growing cat state on one GPU: plain list (reference behaviour: torch.cat of every piece at
every read) vs StateArena (utilities/arena.py).  CatMetric, ``steps`` updates of ``n`` fp32 values, compute() after
every update.  Prints one JSON line."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from torchmetrics_forked_amd import CatMetric  # noqa: E402


def run(steps, n, plain):
    dev = torch.device("cuda", 0)
    m = CatMetric(nan_strategy="error").to(dev)  # NaN check is a device flag, no NaN-drop pass: the list itself is what is measured
    xs = [torch.randn(n, device=dev) for _ in range(16)]
    if plain:
        m.value = []  # a plain list: torch.cat of every piece at every read (the reference's behaviour)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        m.update(xs[i % 16])
        out = m.compute()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3, out.numel()


def main():
    res = {}
    for steps, n in ((1000, 4096), (200, 1 << 20)):
        run(20, n, True)
        run(20, n, False)
        tp, k1 = run(steps, n, True)
        ta, k2 = run(steps, n, False)
        assert k1 == k2 == steps * n
        res[f"steps{steps}_n{n}"] = {"plain_list_ms": round(tp, 1), "arena_ms": round(ta, 1), "speedup": round(tp / ta, 2)}
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
