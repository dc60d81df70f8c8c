"""bert_greedy_match at the BASELINE shape (256 pairs x 512 x 512 x 768, bf16): time and TFLOP/s."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from torchmetrics_forked_amd import ops  # noqa: E402

ops.require()
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
res = {}
for (b, lp, lr, d) in [(256, 512, 512, 768), (1024, 512, 512, 768), (64, 128, 128, 768)]:
    p = torch.nn.functional.normalize(torch.randn(b, lp, d, device=dev, generator=g), dim=-1).bfloat16()
    r = torch.nn.functional.normalize(torch.randn(b, lr, d, device=dev, generator=g), dim=-1).bfloat16()
    for _ in range(3):
        torch.ops.tmx.bert_greedy_match(p, r)
    torch.cuda.synchronize()
    n = 10
    t0 = time.perf_counter()
    for _ in range(n):
        torch.ops.tmx.bert_greedy_match(p, r)
    torch.cuda.synchronize()
    us = (time.perf_counter() - t0) / n * 1e6
    res[f"{b}x{lp}x{lr}x{d}"] = {"us": round(us, 1), "tflops": round(2 * b * lp * lr * d / (us * 1e-6) / 1e12, 1)}
print(json.dumps({"bert_greedy_match_bf16": res}))
