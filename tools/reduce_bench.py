"""Curve-histogram reduce + summary (``tmx::curve_hist_scores``) on the headline's histogram: MulticlassAUROC, C = 1000,
one 65536-row bf16 batch (the occupied code ranges of randn logits).  Times the op (median of 50, CUDA events) for the
block-per-class and the wave-per-class kernel (``TMX_REDUCE_FORM``, one child process each); checks that both
give the same scores.  One JSON line.

    python tools/reduce_bench.py
"""
import json
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def measure() -> dict:
    import torch

    import torchmetrics_forked_amd as tm
    from torchmetrics_forked_amd import ops

    ops.require()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(3)
    m = tm.MulticlassAUROC(num_classes=1000).to(dev)
    m.update(torch.randn(65536, 1000, device=dev, generator=g).bfloat16(), torch.randint(0, 1000, (65536,), device=dev, generator=g))
    hist, rng = m.score_hist, m._tracked_range()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for i in range(60):
        e0.record()
        sc, summ = torch.ops.tmx.curve_hist_scores(hist, rng, False)
        e1.record()
        e1.synchronize()
        if i >= 10:
            ts.append(e0.elapsed_time(e1) * 1e3)
    ts.sort()
    return {"us": round(ts[len(ts) // 2], 2), "scores_sum": float(sc[:, :2].nan_to_num(0).sum()), "summary": [float(v) for v in summ[:8]],
            "auroc": float(m.compute())}


def main() -> None:
    if os.environ.get("REDUCE_BENCH_CHILD"):
        print(json.dumps(measure()), flush=True)
        return
    out = {"what": "tmx::curve_hist_scores (reduce + summary, one launch) on MulticlassAUROC C=1000 after one 65536-row bf16 batch"}
    env = dict(os.environ, REDUCE_BENCH_CHILD="1")
    for name, extra in (("block_per_class", {"TMX_REDUCE_FORM": "block"}), ("wave_per_class", {"TMX_REDUCE_FORM": "wave"})):
        r = subprocess.run([sys.executable, __file__], env={**env, **extra}, capture_output=True, text=True, timeout=300)
        lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
        out[name] = json.loads(lines[-1]) if lines else {"error": r.stderr[-500:]}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
