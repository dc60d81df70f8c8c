"""Measure the reference library (TorchMetrics 1.3.0dev, unmodified source) on the headline config with the
same harness as bench.py: K x ``MetricCollection.update`` + one ``compute`` on bf16 logits [65536, 1000].

The reference source is unpacked from an untracked tarball (``.refbench/ref_src.tar.gz``, never committed) into
a temp dir; ``tests/_oracle`` provides the 4 ``lightning_utilities`` helpers it imports.
Prints one JSON line with ``ref_updates_per_sec``.
"""
import argparse
import json
import os
import sys
import tarfile
import tempfile
import time

import torch


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--tar", default=os.path.join(os.path.dirname(__file__), "..", ".refbench", "ref_src.tar.gz"))
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--num-classes", type=int, default=1000)
    ap.add_argument("--batch", type=int, default=65536)
    args = ap.parse_args()
    tmp = tempfile.mkdtemp(prefix="refsrc_")
    with tarfile.open(args.tar) as tf:
        tf.extractall(tmp)
    root = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [os.path.join(root, "..", "tests", "_oracle"), os.path.join(tmp, "src")]
    import warnings

    warnings.filterwarnings("ignore")
    from torchmetrics import MetricCollection
    from torchmetrics.classification import MulticlassAUROC, MulticlassConfusionMatrix

    dev = torch.device("cuda", 0)
    C, B = args.num_classes, args.batch
    coll = MetricCollection({"auroc": MulticlassAUROC(num_classes=C), "confmat": MulticlassConfusionMatrix(num_classes=C)}).to(dev)
    gen = torch.Generator(device=dev).manual_seed(1234)
    pool = [(torch.randn(B, C, device=dev, generator=gen).to(torch.bfloat16), torch.randint(0, C, (B,), device=dev, generator=gen)) for _ in range(4)]
    for i in range(args.warmup):
        coll.update(*pool[i % 4])
    coll.reset()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        coll.update(*pool[i % 4])
    torch.cuda.synchronize()
    t_upd = time.perf_counter() - t0
    res = coll.compute()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print(json.dumps({
        "ref_updates_per_sec": args.steps / el,
        "ref_ms_per_step": 1000 * el / args.steps,
        "ref_update_only_ms_per_step": 1000 * t_upd / args.steps,
        "ref_compute_ms": 1000 * (el - t_upd),
        "steps": args.steps,
        "auroc": float(res["auroc"]),
    }), flush=True)


if __name__ == "__main__":
    main()
