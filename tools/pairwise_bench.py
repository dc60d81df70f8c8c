"""Fused pairwise GEMM kernel (``torch.ops.tmx.pairwise_gemm``) vs the reference's ATen composition on one GPU:
linear / cosine / euclidean at metric-sized shapes, fp32 and bf16 (fp64 for euclidean's accumulation either way).
Prints one JSON object (median ms over repeats, after warm-up)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    import torch

    from torchmetrics_forked_amd import ops
    from torchmetrics_forked_amd.functional.pairwise import helpers
    import torchmetrics_forked_amd.functional.pairwise as FP

    ops.require()
    fns = {"linear": FP.pairwise_linear_similarity, "cosine": FP.pairwise_cosine_similarity,
           "euclidean": FP.pairwise_euclidean_distance}
    if os.environ.get("PW_MODES"):  # e.g. "linear,cosine"
        fns = {k: v for k, v in fns.items() if k in os.environ["PW_MODES"].split(",")}
    shapes = [(1000, 1000, 128), (4096, 4096, 512), (8192, 8192, 256), (16384, 2048, 1024), (2048, 2048, 4096)]
    if os.environ.get("PW_SHAPES"):  # "N:M:D,N:M:D,..." (crossover sweeps for the routing in functional/pairwise/helpers.py)
        shapes = [tuple(int(v) for v in t.split(":")) for t in os.environ["PW_SHAPES"].split(",")]
    force = os.environ.get("PW_FORCE_FUSED", "1") == "1"  # time the kernel even where the routing would take ATen
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def med_ms(fn, reps=10):
        for _ in range(3):
            fn()
        ts = []
        for _ in range(reps):
            ev0.record()
            fn()
            ev1.record()
            ev1.synchronize()
            ts.append(ev0.elapsed_time(ev1))
        ts.sort()
        return round(ts[len(ts) // 2], 4)

    res = {}
    for (n, m, d) in shapes:
        dtypes = [getattr(torch, t) for t in os.environ.get("PW_DTYPES", "float32,bfloat16").split(",")]
        for dtype in dtypes:
            x = torch.randn(n, d, device="cuda").to(dtype)
            y = torch.randn(m, d, device="cuda").to(dtype)
            for name, fn in fns.items():
                helpers._FUSED = "force" if force else True
                t_fused = med_ms(lambda: fn(x, y))
                helpers._FUSED = False
                t_aten = med_ms(lambda: fn(x, y))
                helpers._FUSED = True
                key = f"{name}_{n}x{m}x{d}_{str(dtype).split('.')[-1]}"
                res[key] = {"fused_ms": t_fused, "aten_ms": t_aten, "speedup": round(t_aten / t_fused, 3)}
                print(key, res[key], flush=True)
            del x, y
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
