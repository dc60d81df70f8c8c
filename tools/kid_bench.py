"""KernelInceptionDistance compute on one GPU: fused per-subset sums (kid_poly_sums: the f16-split matrix-core route for fp32,
and with it switched off the round-5 fp32 MFMA kernel) vs the reference's poly_mmd composition, 2000 real / 2000 fake Inception-2048 features (synthetic), 100 subsets of 1000.  One JSON line (ms)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    import torch

    from torchmetrics_forked_amd import ops
    from torchmetrics_forked_amd.image import generative as G

    ops.require()
    real = torch.randn(2000, 2048, device="cuda")
    fake = torch.randn(2000, 2048, device="cuda") + 0.1
    m, subsets = 1000, 100

    def fused():
        draws = [(torch.randperm(2000)[:m], torch.randperm(2000)[:m]) for _ in range(subsets)]
        s = torch.ops.tmx.kid_poly_sums(real, fake, torch.stack([d[0] for d in draws]), torch.stack([d[1] for d in draws]),
                                        3, 1.0 / 2048, 1.0)
        return ((s[:, 0] + s[:, 1]) / (m * (m - 1)) - 2 * s[:, 2] / m**2).mean()

    def composed():
        out = []
        for _ in range(subsets):
            a = real[torch.randperm(2000)[:m]]
            b = fake[torch.randperm(2000)[:m]]
            out.append(G.poly_mmd(a, b, 3, None, 1.0))
        return torch.stack(out).mean()

    def fused_exact():  # the fp32-MFMA kernel (round 5), the x3 route switched off
        os.environ["TMX_PAIRWISE_X3_OFF"] = "1"
        try:
            return fused()
        finally:
            del os.environ["TMX_PAIRWISE_X3_OFF"]

    res = {}
    for name, fn in (("fused", fused), ("fused_fp32_mfma", fused_exact), ("composed", composed)):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(3):
            torch.manual_seed(0)
            t0 = time.perf_counter()
            v = fn()
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        res[name] = {"ms": round(min(ts), 3), "kid": float(v)}
    res["speedup"] = round(res["composed"]["ms"] / res["fused"]["ms"], 3)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
