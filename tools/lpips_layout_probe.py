"""LPIPS trunk (VGG16, random init, fp32) memory-format probe: the five tapped feature maps of 16 images of
3 x 1024 x 1024 in NCHW (the reference's layout) vs channels_last (MIOpen's NHWC convolutions without its layout
transposes).  One JSON line of median ms per forward."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from torchmetrics_forked_amd.functional.image.lpips import _SlicedBackbone  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(0)
x = torch.rand(16, 3, 1024, 1024, device=dev) * 2 - 1
out = {}
for fmt in ("nchw", "channels_last"):
    net = _SlicedBackbone("vgg").to(dev).eval()
    xin = x
    if fmt == "channels_last":
        net = net.to(memory_format=torch.channels_last)
        xin = x.contiguous(memory_format=torch.channels_last)
    ts = []
    with torch.no_grad():
        for i in range(6):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            feats = net(xin)
            torch.cuda.synchronize()
            if i:
                ts.append(1e3 * (time.perf_counter() - t0))
            del feats
    out[fmt] = round(sorted(ts)[len(ts) // 2], 2)
    print(fmt, out[fmt], flush=True)
print(json.dumps(out), flush=True)
