"""LPIPS(VGG16) trunk layout experiment on one MI355X: the trunk dominates the image config (SSIM+PSNR+LPIPS,
256 x 3 x 1024^2). Times one chunk (16 pairs = 32 images through the trunk) for
  nchw      both inputs as two trunk calls (current default)
  nchw_cat  both inputs as ONE trunk call (one conv launch per layer instead of two)
  nhwc_cat  channels_last weights and inputs, one trunk call
and, last (it changes MIOpen's global algorithm choice), the same with torch.backends.cudnn.benchmark=True.
Prints one JSON line."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from torchmetrics_forked_amd.models.backbones import vgg16_features  # noqa: E402


def timed(fn, steps=3, warmup=1):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    net = vgg16_features().eval().to(dev)
    pairs = int(os.environ.get("PAIRS", "16"))
    a = torch.randn(pairs, 3, 1024, 1024, device=dev)
    b = torch.randn(pairs, 3, 1024, 1024, device=dev)
    out = {"pairs": pairs, "image": "3x1024x1024 fp32"}
    with torch.no_grad():
        ref = net(torch.cat([a[:2], b[:2]]))
        out["nchw_ms"] = round(timed(lambda: (net(a), net(b))), 2)
        print(json.dumps(out), flush=True)
        out["nchw_cat_ms"] = round(timed(lambda: net(torch.cat([a, b]))), 2)
        net_cl = vgg16_features().eval().to(dev)
        net_cl.load_state_dict(net.state_dict())
        net_cl = net_cl.to(memory_format=torch.channels_last)
        ab_cl = torch.cat([a, b]).contiguous(memory_format=torch.channels_last)
        out["nhwc_cat_ms"] = round(timed(lambda: net_cl(ab_cl)), 2)
        got = net_cl(torch.cat([a[:2], b[:2]]).contiguous(memory_format=torch.channels_last))
        out["nhwc_max_rel_diff"] = float(((got - ref).abs().max() / ref.abs().max()))
        print(json.dumps(out), flush=True)
        if os.environ.get("LPIPS_BENCHMARK_MODE", "0") != "1":  # MIOpen exhaustive find at 1024^2 ran > 3 min silent
            print(json.dumps(out), flush=True)
            return
        torch.backends.cudnn.benchmark = True
        t0 = time.perf_counter()
        net(torch.cat([a, b]))
        torch.cuda.synchronize()
        out["bench_first_call_s"] = round(time.perf_counter() - t0, 2)
        out["nchw_cat_benchmark_ms"] = round(timed(lambda: net(torch.cat([a, b]))), 2)
        out["nhwc_cat_benchmark_ms"] = round(timed(lambda: net_cl(ab_cl)), 2)
    flops = 0.0  # conv FLOPs of the trunk per image (2 * Cin * Cout * 9 * H * W per 3x3 conv)
    h = 1024
    for m in net:
        if isinstance(m, torch.nn.Conv2d):
            flops += 2 * m.in_channels * m.out_channels * 9 * h * h
        elif isinstance(m, torch.nn.MaxPool2d):
            h //= 2
    best = min(v for k, v in out.items() if k.endswith("_ms"))
    out["trunk_gflop_per_image"] = round(flops / 1e9, 1)
    out["best_tflops"] = round(flops * 2 * pairs / (best * 1e-3) / 1e12, 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
