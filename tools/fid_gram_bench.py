"""FID moment update on one GPU: the fused in-place ``fid_gram_update`` kernel vs the reference's
``double() + sum + addmm`` at feature batches of the Inception-2048 head.  Prints one JSON object (median us)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    import torch

    from torchmetrics_forked_amd import ops

    ops.require()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def med_us(fn, reps=20):
        for _ in range(3):
            fn()
        ts = []
        for _ in range(reps):
            ev0.record()
            fn()
            ev1.record()
            ev1.synchronize()
            ts.append(ev0.elapsed_time(ev1) * 1e3)
        ts.sort()
        return round(ts[len(ts) // 2], 2)

    res = {}
    for (b, f) in ((256, 2048), (64, 2048), (1024, 2048), (256, 768), (512, 192)):
        for dtype in (torch.float32, torch.float64):
            x = torch.randn(b, f, device="cuda", dtype=dtype)
            gram = torch.zeros(f, f, dtype=torch.float64, device="cuda")
            colsum = torch.zeros(f, dtype=torch.float64, device="cuda")
            state = {"g": gram.clone(), "s": colsum.clone()}

            def ref():
                xd = x.double()
                state["s"] = state["s"] + xd.sum(dim=0)
                state["g"] = state["g"].addmm(xd.t(), xd)

            t_fused = med_us(lambda: torch.ops.tmx.fid_gram_update(x, gram, colsum))
            t_ref = med_us(ref)
            key = f"B{b}_F{f}_{str(dtype).split('.')[-1]}"
            res[key] = {"fused_us": t_fused, "reference_ops_us": t_ref, "speedup": round(t_ref / t_fused, 3)}
            print(key, res[key], flush=True)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
