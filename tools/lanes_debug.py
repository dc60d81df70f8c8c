"""Debug probe for the curve update lanes: single-stream vs two-lane histograms after a few batches, with and without
a softmax-decision flip; prints where they differ.

    python tools/lanes_debug.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    import torch

    import torchmetrics_forked_amd as tm
    from torchmetrics_forked_amd import ops
    from torchmetrics_forked_amd.classification import precision_recall_curve as prc

    ops.require()
    for c, probs_at, k in ((512, (), 2), (512, (), 5), (512, (3,), 5), (1000, (), 5), (1000, (1,), 2)):
        n = (1 << 22) // c + 64
        g = torch.Generator(device="cuda").manual_seed(c)
        bs = []
        for i in range(k):
            x = torch.randn(n, c, device="cuda", generator=g) * 3
            if i in probs_at:
                x = x.softmax(-1)
            bs.append((x.bfloat16(), torch.randint(0, c, (n,), device="cuda", generator=g)))
        hs = []
        for lanes in (False, True):
            prc._LANES_ON = lanes
            m = tm.MulticlassAUROC(num_classes=c).cuda()
            for p, t in bs:
                m.update(p, t)
            h = m.metric_state["score_hist"].clone()
            hs.append((h, m.compute(), m._tracked_range().clone()))
        (h0, a0, r0), (h1, a1, r1) = hs
        diff = (h0 != h1)
        print(f"C={c} batches={k} probs_at={probs_at}: auroc {a0.item():.9f} vs {a1.item():.9f}; hist equal {bool(not diff.any())};"
              f" total {int(h0.sum())} vs {int(h1.sum())}; neg {int(h0[:, 0].sum())} vs {int(h1[:, 0].sum())};"
              f" pos {int(h0[:, 1].sum())} vs {int(h1[:, 1].sum())}; range equal {torch.equal(r0, r1)}", flush=True)
        if diff.any():
            idx = diff.nonzero()[:8].tolist()
            print("   first diffs (class, neg/pos, code):", idx, [(int(h0[tuple(i)]), int(h1[tuple(i)])) for i in idx], flush=True)
            print("   classes differing:", int(diff.any(-1).any(-1).sum()), flush=True)


if __name__ == "__main__":
    main()
