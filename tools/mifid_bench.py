"""MiFID memorization term on one GPU: fused row maxima of |cos| (pairwise_abs_cos_rowmax) vs the reference's
normalise / matmul / abs / min composition, synthetic fp32 features at four sizes.  One JSON line (ms)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    import torch

    from torchmetrics_forked_amd import ops

    ops.require()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    a = b = None

    def fused():
        return torch.mean(1.0 - torch.ops.tmx.pairwise_abs_cos_rowmax(a, b))

    def composed():
        n1 = a / torch.norm(a, dim=1, keepdim=True)
        n2 = b / torch.norm(b, dim=1, keepdim=True)
        return torch.mean((1.0 - torch.abs(n1 @ n2.t())).min(dim=1).values)

    out = {}
    for (n, d) in ((10000, 2048), (2000, 512), (1000, 2048), (4000, 256)):
        a = torch.randn(n, d, device="cuda")
        b = torch.randn(n, d, device="cuda")
        res = {}
        for name, fn in (("fused", fused), ("composed", composed)):
            fn()
            ts = []
            for _ in range(5):
                ev0.record()
                v = fn()
                ev1.record()
                ev1.synchronize()
                ts.append(ev0.elapsed_time(ev1))
            res[name] = {"ms": round(sorted(ts)[2], 3), "value": float(v)}
        res["speedup"] = round(res["composed"]["ms"] / res["fused"]["ms"], 3)
        out[f"{n}x{n}x{d}"] = res
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
