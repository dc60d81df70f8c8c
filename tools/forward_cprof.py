"""Host profile of the headline collection's GPU ``forward`` (MulticlassAUROC + MulticlassConfusionMatrix, C = 1000,
65536 bf16 rows): cProfile over 50 forwards after warm-up, the top functions by cumulative and by self time (us per
forward).  Complements tools/forward_bench.py (device timeline) for the host-enqueue side.

    python tools/forward_cprof.py
"""
import cProfile
import io
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    import torch

    import torchmetrics_forked_amd as tm
    from torchmetrics_forked_amd import ops

    ops.require()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(7)
    pool = [(torch.randn(65536, 1000, device=dev, generator=g).bfloat16(), torch.randint(0, 1000, (65536,), device=dev, generator=g)) for _ in range(4)]
    coll = tm.MetricCollection({"auroc": tm.MulticlassAUROC(num_classes=1000), "confmat": tm.MulticlassConfusionMatrix(num_classes=1000)}).to(dev)
    for i in range(10):
        coll(*pool[i % 4])
    torch.cuda.synchronize(dev)
    steps = 50
    pr = cProfile.Profile()
    pr.enable()
    for i in range(steps):
        coll(*pool[i % 4])
    pr.disable()
    torch.cuda.synchronize(dev)
    for key in ("cumulative", "tottime"):
        s = io.StringIO()
        st = pstats.Stats(pr, stream=s).sort_stats(key)
        st.print_stats(35)
        print(f"--- forward: by {key} (totals over {steps} forwards)")
        print(s.getvalue()[:9000])


if __name__ == "__main__":
    main()
