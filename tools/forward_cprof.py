"""Host profile of the headline collection's GPU ``forward`` (MulticlassAUROC + MulticlassConfusionMatrix, C = 1000,
65536 bf16 rows): cProfile over 50 forwards after warm-up, the top functions by cumulative and by self time (us per
forward).  Complements tools/forward_bench.py (device timeline) for the host-enqueue side.

    python tools/forward_cprof.py
"""
import cProfile
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
    import time

    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(steps):
        coll(*pool[i % 4])
    t1 = time.perf_counter()
    torch.cuda.synchronize(dev)
    t_upd = time.perf_counter()
    for i in range(steps):
        coll.update(*pool[i % 4])
    t_upd1 = time.perf_counter()
    torch.cuda.synchronize(dev)
    print(f"host enqueue without profiler: forward {1e6 * (t1 - t0) / steps:.1f} us, update {1e6 * (t_upd1 - t_upd) / steps:.1f} us "
          "(queue-bound once the device falls behind: compare the two)")
    pr = cProfile.Profile()
    pr.enable()
    for i in range(steps):
        coll(*pool[i % 4])
    pr.disable()
    torch.cuda.synchronize(dev)
    st = pstats.Stats(pr).stats
    print(f"--- forward: by cumulative (us per forward, cProfile on), {sum(v[1] for v in st.values()) / steps:.0f} calls per forward")
    for ct, tt, nc, k in sorted(((v[3], v[2], v[1], k) for k, v in st.items()), reverse=True)[:45]:
        print(f"{1e6 * ct / steps:10.1f} {1e6 * tt / steps:10.1f} {nc:8d} {os.path.basename(k[0])}:{k[1]}({k[2]})")
    print("--- forward: by self time")
    for tt, ct, nc, k in sorted(((v[2], v[3], v[1], k) for k, v in st.items()), reverse=True)[:45]:
        print(f"{1e6 * tt / steps:10.1f} {1e6 * ct / steps:10.1f} {nc:8d} {os.path.basename(k[0])}:{k[1]}({k[2]})")

if __name__ == "__main__":
    main()
