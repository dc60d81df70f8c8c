"""Secondary BASELINE configs on one MI355X (BASELINE.json "configs" 3-5), ours vs the reference where the
reference can run in this image (its MAP needs pycocotools and its LPIPS needs torchvision: not installed).

* map       MeanAveragePrecision, COCO-80 synthetic, 512 images / step, 100 detections + 20 ground truths per image
* image     SSIM + PSNR on 3x1024x1024, bs=256 (reference: same metrics, unmodified source); LPIPS (random-init
            VGG16, fused head kernel) at bs=32 per call
* bert      BERTScore with random-init bert-base, 512-token pairs, bs=1024 (ours); reference at bs=64 (it moves
            embeddings to the CPU and scores there, so its full-size run would dominate the GPU budget)

Prints one JSON line per config.  Timings bracket ``torch.cuda.synchronize()``.
"""
import argparse
import json
import os
import sys
import tarfile
import tempfile
import time

import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)


def _timed(fn, steps, warmup):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def _reference():
    tar = os.path.join(ROOT, ".refbench", "ref_src.tar.gz")
    if not os.path.exists(tar):
        return None
    tmp = tempfile.mkdtemp(prefix="refsrc_")
    with tarfile.open(tar) as tf:
        tf.extractall(tmp)
    sys.path[:0] = [os.path.join(ROOT, "tests", "_oracle"), os.path.join(tmp, "src")]
    import warnings

    warnings.filterwarnings("ignore")
    import torchmetrics

    return torchmetrics


def bench_map(dev, steps, warmup):
    from torchmetrics_forked_amd.detection import MeanAveragePrecision

    g = torch.Generator(device=dev).manual_seed(0)
    n_img, n_det, n_gt, n_cls = 512, 100, 20, 80

    def batch():
        xy = torch.rand(n_img, n_gt, 2, device=dev, generator=g) * 500
        gt = torch.cat([xy, xy + torch.rand(n_img, n_gt, 2, device=dev, generator=g) * 150 + 4], -1)
        det = torch.cat([gt + torch.randn(n_img, n_gt, 4, device=dev, generator=g) * 6,
                         torch.cat([xy, xy + 50], -1)[:, torch.randint(0, n_gt, (n_det - n_gt,), device=dev, generator=g)] + 30], 1)
        det[..., 2:] = torch.maximum(det[..., 2:], det[..., :2] + 1)
        gl = torch.randint(0, n_cls, (n_img, n_gt), device=dev, generator=g)
        dl = torch.cat([gl, torch.randint(0, n_cls, (n_img, n_det - n_gt), device=dev, generator=g)], 1)
        sc = torch.rand(n_img, n_det, device=dev, generator=g)
        preds = [{"boxes": det[i], "scores": sc[i], "labels": dl[i]} for i in range(n_img)]
        target = [{"boxes": gt[i], "labels": gl[i]} for i in range(n_img)]
        return preds, target

    data = [batch() for _ in range(2)]
    m = MeanAveragePrecision().to(dev)
    t_update = _timed(lambda: m.update(*data[0]), steps, warmup)
    m.reset()
    for p, t in data:
        m.update(p, t)
    t0 = time.perf_counter()
    res = m.compute()
    t_compute = time.perf_counter() - t0
    return {"config": "MeanAveragePrecision COCO-80 synthetic 512 img/step x 100 det", "update_ms": round(t_update * 1e3, 2),
            "images_per_sec_update": round(n_img / t_update, 1), "compute_s_1024_images": round(t_compute, 3),
            "map": round(float(res["map"]), 4)}


def bench_image(dev, steps, warmup, ref):
    from torchmetrics_forked_amd.image import LearnedPerceptualImagePatchSimilarity, PeakSignalNoiseRatio, StructuralSimilarityIndexMeasure

    b = 256
    g = torch.Generator(device=dev).manual_seed(0)
    t = torch.rand(b, 3, 1024, 1024, device=dev, generator=g)
    p = (t + 0.05 * torch.randn(b, 3, 1024, 1024, device=dev, generator=g)).clamp(0, 1)
    out = {"config": "SSIM + PSNR 3x1024x1024 bs=256 fp32; LPIPS(random VGG16) bs=32"}
    ssim, psnr = StructuralSimilarityIndexMeasure(data_range=1.0).to(dev), PeakSignalNoiseRatio(data_range=1.0).to(dev)
    out["ours_ssim_psnr_ms"] = round(_timed(lambda: (ssim.update(p, t), psnr.update(p, t)), steps, warmup) * 1e3, 2)
    if ref is not None:
        rs = ref.image.StructuralSimilarityIndexMeasure(data_range=1.0).to(dev)
        rp = ref.image.PeakSignalNoiseRatio(data_range=1.0).to(dev)
        try:
            out["ref_ssim_psnr_ms"] = round(_timed(lambda: (rs.update(p, t), rp.update(p, t)), max(1, steps // 2), 1) * 1e3, 2)
            out["speedup_ssim_psnr"] = round(out["ref_ssim_psnr_ms"] / out["ours_ssim_psnr_ms"], 2)
        except torch.cuda.OutOfMemoryError:
            out["ref_ssim_psnr_ms"] = "OOM"
        del rs, rp
        torch.cuda.empty_cache()
    lp = LearnedPerceptualImagePatchSimilarity(net_type="vgg", normalize=True).to(dev)
    pl, tl = p[:32], t[:32]
    out["ours_lpips_bs32_ms"] = round(_timed(lambda: lp.update(pl, tl), max(1, steps // 2), 1) * 1e3, 2)
    return out


def bench_bert(dev, steps, warmup, ref):
    import transformers

    from torchmetrics_forked_amd.functional.text import bert_score

    cfg = transformers.BertConfig()  # bert-base geometry, random init
    torch.manual_seed(0)
    model = transformers.BertModel(cfg).eval().to(dev).to(torch.bfloat16)
    n, L = 1024, 512
    g = torch.Generator().manual_seed(0)
    ids_p = torch.randint(1000, 30000, (n, L), generator=g)
    ids_t = torch.randint(1000, 30000, (n, L), generator=g)
    mask = torch.ones(n, L, dtype=torch.long)
    preds = {"input_ids": ids_p, "attention_mask": mask}
    target = {"input_ids": ids_t, "attention_mask": mask}
    run = lambda: bert_score(preds, target, model=model, batch_size=128, device=dev)  # noqa: E731
    t_all = _timed(run, max(1, steps // 4), 1)
    # greedy-matching kernel alone on embeddings of the same shape
    p = torch.nn.functional.normalize(torch.randn(n, L, 768, device=dev), dim=-1).bfloat16()
    r = torch.nn.functional.normalize(torch.randn(n, L, 768, device=dev), dim=-1).bfloat16()
    t_k = _timed(lambda: torch.ops.tmx.bert_greedy_match(p, r), steps, warmup)
    out = {"config": "BERTScore random-init bert-base bf16, 512-token pairs, bs=1024", "ours_pairs_per_sec": round(n / t_all, 1),
           "ours_total_s": round(t_all, 3), "greedy_match_kernel_ms": round(t_k * 1e3, 3),
           "greedy_match_tflops": round(2 * n * L * L * 768 / t_k / 1e12, 1)}
    if ref is not None:
        from torchmetrics.functional.text import bert_score as ref_bs

        k = 32
        sub_p = {"input_ids": ids_p[:k], "attention_mask": mask[:k]}
        sub_t = {"input_ids": ids_t[:k], "attention_mask": mask[:k]}
        t_ref = _timed(lambda: ref_bs(sub_p, sub_t, model=model, batch_size=64, device=dev), 1, 0)
        out["ref_pairs_per_sec_bs32"] = round(k / t_ref, 1)
        out["speedup_pairs_per_sec"] = round(out["ours_pairs_per_sec"] / out["ref_pairs_per_sec_bs32"], 1)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--which", default="map,image,bert")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--no-ref", action="store_true")
    args = ap.parse_args()
    from torchmetrics_forked_amd import ops

    ops.require()
    dev = torch.device("cuda", 0)
    ref = None if args.no_ref else _reference()
    for w in args.which.split(","):
        if w == "map":
            res = bench_map(dev, args.steps, args.warmup)
        elif w == "image":
            res = bench_image(dev, args.steps, args.warmup, ref)
        elif w == "bert":
            res = bench_bert(dev, args.steps, args.warmup, ref)
        else:
            continue
        print(json.dumps(res), flush=True)
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
