"""fp32 / fp64 exact curves through the hand-written radix engine (csrc/radix.hip) vs the bf16 exact histogram.

Prints one JSON object: BinaryAUROC / BinaryAveragePrecision at N = 16.7M (50% positives) update + compute for
fp32 and bf16 scores, and MulticlassAUROC fp32 65536 x 1000 after K updates (compute time; > 8192 positives per
class once K > 125, i.e. past the anchored kernel's window).
Usage: python tools/radix_curve_bench.py [--mc-steps K]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import torchmetrics_forked_amd as tm  # noqa: E402
from torchmetrics_forked_amd import ops  # noqa: E402


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return best


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--mc-steps", type=int, default=20)
    args = ap.parse_args()
    ops.require()
    dev = torch.device("cuda", 0)
    out = {}
    N = 1 << 24
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.rand(N, device=dev, generator=g)
    t = (torch.rand(N, device=dev, generator=g) < 0.5).long()
    for name, cls in (("BinaryAUROC", tm.BinaryAUROC), ("BinaryAveragePrecision", tm.BinaryAveragePrecision)):
        for dt in (torch.float32, torch.bfloat16):
            xd = x.to(dt)

            def run():
                m = cls().to(dev)
                m.update(xd, t)
                return m.compute()

            out[f"{name}_{str(dt).split('.')[-1]}_N{N}_update_compute_ms"] = round(1e3 * timed(run), 3)
        out[f"{name}_fp32_over_bf16"] = round(out[f"{name}_float32_N{N}_update_compute_ms"] / out[f"{name}_bfloat16_N{N}_update_compute_ms"], 2)
    C, B = 1000, 65536
    m = tm.MulticlassAUROC(num_classes=C).to(dev)
    pool = [torch.randn(B, C, device=dev, generator=g) for _ in range(2)]
    tgt = torch.randint(0, C, (B,), device=dev, generator=g)
    for i in range(args.mc_steps):
        m.update(pool[i % 2], tgt)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    v = m.compute()
    torch.cuda.synchronize()
    out[f"MulticlassAUROC_fp32_C{C}_B{B}_x{args.mc_steps}_compute_ms"] = round(1e3 * (time.perf_counter() - t0), 2)
    out["mc_auroc"] = float(v)
    out["samples_per_class"] = B * args.mc_steps
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
