"""Same-shape comparisons of the secondary BASELINE configs against the unmodified reference, on one MI355X.

Both sides get the SAME inputs, the SAME model object and the SAME batch size:

* ``bert``  BERTScore, random-init bert-base in bf16, 1024 pairs x 512 tokens, ``batch_size=128`` (reference:
  ``torchmetrics.functional.text.bert_score`` with ``model=`` the same module).
* ``image`` SSIM (gaussian 11x11) + PSNR on 256 x 3 x 1024 x 1024 fp32 (reference modules, unmodified).
  LPIPS is not compared: the reference's LPIPS needs torchvision, which is not installed.
* ``map``   not compared: the reference's MeanAveragePrecision needs pycocotools / faster-coco-eval or torchvision.

The reference source comes from ``.refbench/ref_src.tar.gz`` (untracked; ``tools/make_refbench.sh`` builds it from
the reference checkout). Prints one JSON line per config.
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

from domain_bench import _reference  # noqa: E402


def _timed(fn, steps, warmup):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def bench_bert(dev, ref, steps):
    import transformers

    from torchmetrics_forked_amd.functional.text import bert_score

    torch.manual_seed(0)
    model = transformers.BertModel(transformers.BertConfig()).eval().to(dev).to(torch.bfloat16)
    n, L, bs = 1024, 512, 128
    g = torch.Generator().manual_seed(0)
    ids_p = torch.randint(1000, 30000, (n, L), generator=g)
    ids_t = torch.randint(1000, 30000, (n, L), generator=g)
    mask = torch.ones(n, L, dtype=torch.long)
    preds = {"input_ids": ids_p, "attention_mask": mask}
    target = {"input_ids": ids_t, "attention_mask": mask}
    ours = _timed(lambda: bert_score(preds, target, model=model, batch_size=bs, device=dev), steps, 1)
    out = {"config": "BERTScore random-init bert-base bf16, 1024 pairs x 512 tokens, batch_size=128 (both sides)",
           "ours_s": round(ours, 3), "ours_pairs_per_sec": round(n / ours, 1)}
    if ref is not None:
        from torchmetrics.functional.text import bert_score as ref_bs

        t = _timed(lambda: ref_bs(preds, target, model=model, batch_size=bs, device=dev), steps, 1)
        out.update({"ref_s": round(t, 3), "ref_pairs_per_sec": round(n / t, 1), "speedup": round(t / ours, 2)})
        # same pair order on both sides only when every sentence has the same length (the reference sorts each side
        # by length independently; here every row is 512 tokens, so the pairings agree)
        f_ours = bert_score(preds, target, model=model, batch_size=bs, device=dev)["f1"].float().cpu()
        f_ref = ref_bs(preds, target, model=model, batch_size=bs, device=dev)["f1"].float().cpu()
        out["max_abs_f1_diff"] = float((f_ours - f_ref).abs().max())
        # the reference length-sorts each side on its own (argsort of equal lengths is not stable on the GPU), so
        # its scores can belong to other pairs: match every reference score to the nearest of ours
        out["max_abs_f1_diff_nearest_pair"] = float((f_ref[:, None] - f_ours[None, :]).abs().min(dim=1).values.max())
        out["mean_f1_ours_ref"] = [float(f_ours.mean()), float(f_ref.mean())]
    return out


def bench_image(dev, ref, steps):
    from torchmetrics_forked_amd.image import PeakSignalNoiseRatio, StructuralSimilarityIndexMeasure

    b = 256
    g = torch.Generator(device=dev).manual_seed(0)
    t = torch.rand(b, 3, 1024, 1024, device=dev, generator=g)
    p = (t + 0.05 * torch.randn(b, 3, 1024, 1024, device=dev, generator=g)).clamp(0, 1)
    ssim, psnr = StructuralSimilarityIndexMeasure(data_range=1.0).to(dev), PeakSignalNoiseRatio(data_range=1.0).to(dev)
    ours = _timed(lambda: (ssim.update(p, t), psnr.update(p, t)), steps, 1)
    out = {"config": "SSIM(gaussian 11x11) + PSNR, 256 x 3 x 1024 x 1024 fp32 per update (both sides)",
           "ours_ms": round(ours * 1e3, 2), "ours_images_per_sec": round(b / ours, 1)}
    vals = (float(ssim.compute()), float(psnr.compute()))
    del ssim, psnr
    torch.cuda.empty_cache()
    if ref is not None:
        rs = ref.image.StructuralSimilarityIndexMeasure(data_range=1.0).to(dev)
        rp = ref.image.PeakSignalNoiseRatio(data_range=1.0).to(dev)
        try:
            tr = _timed(lambda: (rs.update(p, t), rp.update(p, t)), steps, 1)
            out.update({"ref_ms": round(tr * 1e3, 2), "ref_images_per_sec": round(b / tr, 1), "speedup": round(tr / ours, 2),
                        "ssim_abs_diff": abs(vals[0] - float(rs.compute())), "psnr_abs_diff": abs(vals[1] - float(rp.compute()))})
        except torch.cuda.OutOfMemoryError:
            out["ref_ms"] = "OOM"
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--which", default="bert,image")
    ap.add_argument("--steps", type=int, default=2)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    ref = _reference()
    for w in args.which.split(","):
        res = {"bert": bench_bert, "image": bench_image}[w](dev, ref, args.steps)
        res["reference_loaded"] = ref is not None
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
