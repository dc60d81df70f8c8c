"""First update of a fresh exact-histogram metric (the speculated normalisation mode has no history yet): GPU time of
that update vs a steady-state update, headline shape (65536 x 1000 bf16 logits).  Prints one JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    import torch

    import torchmetrics_forked_amd as tm

    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(65536, 1000, device=dev, generator=g).bfloat16()
    t = torch.randint(0, 1000, (65536,), device=dev, generator=g)
    warm = tm.MulticlassAUROC(num_classes=1000).to(dev)
    for _ in range(3):
        warm.update(x, t)
    torch.cuda.synchronize(dev)

    def timed(m):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        m.update(x, t)
        b.record()
        b.synchronize()
        return a.elapsed_time(b)

    firsts = []
    for _ in range(3):
        m = tm.MulticlassAUROC(num_classes=1000).to(dev)
        firsts.append(timed(m))
    steady = [timed(m) for _ in range(5)]
    print(json.dumps({"first_update_ms": [round(v, 3) for v in firsts], "steady_update_ms": [round(v, 3) for v in steady]}), flush=True)


if __name__ == "__main__":
    main()
