"""Per-call GPU time of the multiclass pair-stream kernels (confusion matrix vs fused stat scores)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from torchmetrics_forked_amd import ops  # noqa: E402

ops.require()
out = {}
for C, N in ((1000, 65536), (100, 65536), (10, 1 << 20)):
    x = torch.randn(N, C, device="cuda").bfloat16()
    t = torch.randint(0, C, (N,), device="cuda")
    cm = torch.zeros(C, C, dtype=torch.long, device="cuda")
    st = [torch.zeros(C, dtype=torch.long, device="cuda") for _ in range(4)]
    s1 = [torch.zeros(1, dtype=torch.long, device="cuda") for _ in range(4)]
    tk = torch.zeros(9 * 16, dtype=torch.long, device="cuda")
    cases = {
        "confmat": lambda: torch.ops.tmx.mc_confmat_update(x, t, cm, -1, False),
        "stat_macro": lambda: torch.ops.tmx.mc_stat_scores_update(x, t, C, *st, tk, -1, False, False),
        "stat_micro": lambda: torch.ops.tmx.mc_stat_scores_update(x, t, C, *s1, tk, -1, False, True),
    }
    for name, fn in cases.items():
        for _ in range(5):
            fn()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record()
        for _ in range(50):
            fn()
        b.record()
        torch.cuda.synchronize()
        out[f"{name}_C{C}_N{N}"] = round(a.elapsed_time(b) / 50 * 1000, 1)
print(json.dumps({"cap": os.environ.get("TMX_PAIRS_CAP", "1"), "us_per_call": out}))

# binary / multilabel one-launch stats
from torchmetrics_forked_amd.ops import classification as K  # noqa: E402

bout = {}
for name, shape, L, dt in (("binary_16M_fp32", (1 << 24,), 1, torch.float32), ("multilabel_16384x1000_bf16", (16384, 1000), 1000, torch.bfloat16),
                           ("multilabel_65536x16_fp32", (65536, 16), 16, torch.float32)):
    p = torch.rand(shape, device="cuda").to(dt)
    t = torch.randint(0, 2, shape, device="cuda")
    st = tuple(torch.zeros(L, dtype=torch.long, device="cuda") for _ in range(4))
    sc = torch.zeros(6 * L + K.GRID_SLOTS, dtype=torch.long, device="cuda")
    fn = lambda: K.binary_stats_fused(p, t, st, sc, L, 0.5, None)  # noqa: E731
    for _ in range(5):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(50):
        fn()
    b.record()
    torch.cuda.synchronize()
    us = a.elapsed_time(b) / 50 * 1000
    nbytes = p.numel() * p.element_size() + t.numel() * 8
    bout[name] = {"us": round(us, 1), "GBps": round(nbytes / us / 1e3, 1)}
print(json.dumps({"binary_stats_fused": bout}))
