"""Kernel microbenchmarks for the non-classification HIP kernels at BASELINE-like shapes (HIP-event timing).

Run under ``rocprofv3 --kernel-trace --stats`` to get per-kernel device time; prints one JSON line."""
import json
import sys

import torch

sys.path.insert(0, ".")
from torchmetrics_forked_amd import ops  # noqa: E402


def timeit(fn, iters=10, warmup=2):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return round(a.elapsed_time(b) / iters * 1000.0, 1)  # us


def main():
    ops.require()
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    res = {}
    # detection
    xy = torch.rand(4096, 2, device=dev, generator=g) * 800
    boxes = torch.cat([xy, xy + 50], 1)
    for mode in range(4):
        res[f"box_pairwise_mode{mode}_4096x4096_us"] = timeit(lambda: torch.ops.tmx.box_pairwise(boxes, boxes, mode))
    dm = torch.rand(100, 480 * 640, device=dev, generator=g) < 0.3
    from torchmetrics_forked_amd.detection._mask_utils import pack_bits

    db, gb = pack_bits(dm.view(100, 480, 640)), pack_bits(dm[:20].view(20, 480, 640))
    area = dm.sum(1).double()
    res["mask_iou_100x20_480x640_us"] = timeit(lambda: torch.ops.tmx.mask_iou(db, gb, area, area[:20], torch.zeros(20, dtype=torch.bool, device=dev)))
    # text
    logits = torch.randn(8 * 512, 30522, device=dev, generator=g).bfloat16()
    tgt = torch.randint(0, 30522, (8 * 512,), device=dev, generator=g)
    res["token_nll_4096x30522_bf16_us"] = timeit(lambda: torch.ops.tmx.token_nll(logits, tgt, 0, False))
    p = torch.nn.functional.normalize(torch.randn(256, 512, 768, device=dev, generator=g), dim=-1).bfloat16()
    r = torch.nn.functional.normalize(torch.randn(256, 512, 768, device=dev, generator=g), dim=-1).bfloat16()
    t = timeit(lambda: torch.ops.tmx.bert_greedy_match(p, r))
    res["bert_greedy_match_256x512x512x768_bf16_us"] = t
    res["bert_greedy_match_tflops"] = round(2 * 256 * 512 * 512 * 768 / (t * 1e-6) / 1e12, 1)
    # audio
    rr = torch.rand(512, 512, device=dev, dtype=torch.float64, generator=g)
    rr[:, 0] += 512
    bb = torch.rand(512, 512, device=dev, dtype=torch.float64, generator=g)
    res["toeplitz_solve_512sys_L512_us"] = timeit(lambda: torch.ops.tmx.toeplitz_solve(rr, bb))
    x = torch.randn(23 * 64, 16000, device=dev, dtype=torch.float64, generator=g)
    bq = torch.tensor([[1.0, 0.5, 0.2]], device=dev, dtype=torch.float64).expand(23 * 64, 3).contiguous()
    aq = torch.tensor([[1.0, -0.5, 0.1]], device=dev, dtype=torch.float64).expand(23 * 64, 3).contiguous()
    res["iir_filter_1472ch_16000_us"] = timeit(lambda: torch.ops.tmx.iir_filter(x, bq, aq))
    # image / regression / pairwise
    img = torch.rand(16, 3, 1024, 1024, device=dev, generator=g)
    from torchmetrics_forked_amd.functional.image import structural_similarity_index_measure as ssim

    res["ssim_16x3x1024x1024_us"] = timeit(lambda: ssim(img, img * 0.9, data_range=1.0))
    a = torch.randn(1 << 24, 1, device=dev, generator=g)
    res["regression_sums_16M_us"] = timeit(lambda: torch.ops.tmx.regression_sums(a, a * 0.5, 0, 0.0))
    xa = torch.randn(4096, 256, device=dev, generator=g)
    res["pairwise_l1_4096x4096x256_us"] = timeit(lambda: torch.ops.tmx.pairwise_lp(xa, xa, 1.0, False))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
