"""Headroom probe for overlapping the curve update's row pass and class pass: two independent MulticlassAUROC
(C = 1000, 65536 bf16 rows) updates issued back to back on ONE stream vs the same updates split over TWO streams (one
metric per stream, so no state is shared).  If the two-stream per-update time is well below the one-stream time, the
row pass (VALU-bound) and the class pass (memory-bound) of different batches can share the chip.  One JSON line.

    python tools/overlap_probe.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    import torch

    import torchmetrics_forked_amd as tm
    from torchmetrics_forked_amd import ops

    ops.require()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(11)
    pool = [(torch.randn(65536, 1000, device=dev, generator=g).bfloat16(), torch.randint(0, 1000, (65536,), device=dev, generator=g))
            for _ in range(4)]
    ms = [tm.MulticlassAUROC(num_classes=1000).to(dev) for _ in range(2)]
    s = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    steps = 40

    def one_stream() -> float:
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(steps):
            ms[i % 2].update(*pool[i % 4])
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) * 1e3 / steps

    def two_streams() -> float:
        torch.cuda.synchronize(dev)
        cur = torch.cuda.current_stream(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for st in s:
            st.wait_stream(cur)
        for i in range(steps):
            with torch.cuda.stream(s[i % 2]):
                ms[i % 2].update(*pool[i % 4])
        for st in s:
            cur.wait_stream(st)
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) * 1e3 / steps

    for _ in range(3):
        one_stream()
        two_streams()
    a = sorted(one_stream() for _ in range(5))[2]
    b = sorted(two_streams() for _ in range(5))[2]
    print(json.dumps({"what": "MulticlassAUROC C=1000 65536x bf16 update, us per update", "one_stream_us": round(a, 1),
                      "two_streams_us": round(b, 1), "overlap_gain": round(a / b, 3)}), flush=True)


if __name__ == "__main__":
    main()
