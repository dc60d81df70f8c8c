"""In-tree stable radix sort (``ops.sort.sort`` -> ``tmx::radix_sort``) vs ``torch.sort(stable=True)`` on one GPU.

    python tools/sort_bench.py     # one JSON line: per case, median ms of both and the ratio
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    import torch

    from torchmetrics_forked_amd import ops
    from torchmetrics_forked_amd.ops.sort import sort

    ops.require()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    cases = {
        "f32_16.7M": torch.rand(1 << 24, device=dev, generator=g),
        "f32_1M": torch.randn(1 << 20, device=dev, generator=g),
        "f64_4M": torch.randn(1 << 22, device=dev, generator=g, dtype=torch.float64),
        "i64_4M_small_range": torch.randint(0, 1000, (1 << 22,), device=dev, generator=g),
        "i32_4M": torch.randint(-(1 << 30), 1 << 30, (1 << 22,), device=dev, generator=g, dtype=torch.int32),
        "f32_rows_64x262144": torch.randn(64, 1 << 18, device=dev, generator=g),
        "f32_64K": torch.randn(1 << 16, device=dev, generator=g),
        "f32_4K": torch.randn(4096, device=dev, generator=g),
        "f32_rows_256x2048": torch.randn(256, 2048, device=dev, generator=g),
    }

    if os.environ.get("SORT_BENCH_SWEEP"):  # crossover sweep against torch.sort (sets ops/sort.py's routing)
        cases = {}
        for n in (8192, 16384, 32768, 65536, 131072, 196608, 262144, 393216, 524288, 1 << 20):
            cases[f"f32_{n}"] = torch.randn(n, device=dev, generator=g)
            cases[f"i64_{n}"] = torch.randint(-(1 << 40), 1 << 40, (n,), device=dev, generator=g)
        for n in (65536, 262144, 1 << 20, 1 << 22, 1 << 24):
            cases[f"f64_{n}"] = torch.randn(n, device=dev, generator=g, dtype=torch.float64)
        for rows, n in ((4, 65536), (16, 16384), (64, 8192)):
            cases[f"f32_rows_{rows}x{n}"] = torch.randn(rows, n, device=dev, generator=g)
        native = torch.ops.tmx.radix_sort
        sort = lambda x: native(x, False)  # noqa: E731  (the kernel itself, not the routing wrapper)

    def med_ms(fn, reps=15):
        for _ in range(3):
            fn()
        torch.cuda.synchronize(dev)
        ts = []
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            b.record()
            b.synchronize()
            ts.append(a.elapsed_time(b))
        ts.sort()
        return ts[len(ts) // 2]

    out = {}
    for name, x in cases.items():
        ours = med_ms(lambda: sort(x))
        ref = med_ms(lambda: torch.sort(x, dim=-1, stable=True))
        out[name] = {"radix_ms": round(ours, 4), "torch_sort_ms": round(ref, 4), "speedup": round(ref / ours, 2)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
