"""Which fp32 summation order does ATen's GPU softmax use for bf16 rows of 1000 classes?  Emulate candidate orders
with elementwise fp32 ops (each add is one IEEE rounding) and count bit mismatches against torch.softmax."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch

torch.manual_seed(0)
dev = torch.device("cuda", 0)
N, C = 8192, 1000
x = torch.randn(N, C, device=dev).bfloat16()
ref = torch.softmax(x, dim=1)
xf = x.float()
mx = xf.amax(1, keepdim=True)
e = torch.exp(xf - mx)
pad = torch.zeros(N, 1024 - C, device=dev)
ep = torch.cat([e, pad], 1)
res = {}


def finish(s, name):
    q = (e / s).bfloat16()
    res[name] = int((q.view(torch.int16) != ref.view(torch.int16)).sum())
    qm = (e * (1.0 / s)).bfloat16()
    res[name + "_mulrecip"] = int((qm.view(torch.int16) != ref.view(torch.int16)).sum())


# ATen persistent warp softmax, WARP_SIZE 64: lane l sums columns it*64+l sequentially, then xor butterfly 32..1
v = ep.view(N, 16, 64)
s = v[:, 0].clone()
for it in range(1, 16):
    s = s + v[:, it]
for off in (32, 16, 8, 4, 2, 1):
    idx = torch.arange(64, device=dev) ^ off
    s = s + s[:, idx]
finish(s[:, :1], "warp64_seq_xor_desc")
s2 = v[:, 0].clone()
for it in range(1, 16):
    s2 = s2 + v[:, it]
for off in (1, 2, 4, 8, 16, 32):
    idx = torch.arange(64, device=dev) ^ off
    s2 = s2 + s2[:, idx]
finish(s2[:, :1], "warp64_seq_xor_asc")
# warp 32 variant
v32 = ep.view(N, 32, 32)
s3 = v32[:, 0].clone()
for it in range(1, 32):
    s3 = s3 + v32[:, it]
for off in (16, 8, 4, 2, 1):
    idx = torch.arange(32, device=dev) ^ off
    s3 = s3 + s3[:, idx]
finish(s3[:, :1], "warp32_seq_xor_desc")
finish(e.sum(1, keepdim=True), "torch_sum")
finish(e.double().sum(1, keepdim=True).float(), "exact_sum")
# our fused kernel: codes through the curve histogram vs ATen's codes
from torchmetrics_forked_amd.ops import classification as K  # noqa: E402

t = torch.randint(0, C, (N,), device=dev)
hist = torch.zeros(C, 2, K.N_CODES, dtype=torch.long, device=dev)
K.curve_hist_update(x, t, hist, "multiclass", None)
href = torch.zeros_like(hist)
codes = ref.view(torch.int16).long() & 0x3FFF
lab = (torch.arange(C, device=dev)[None, :] == t[:, None]).long()
flat = (torch.arange(C, device=dev)[None, :] * 2 + lab) * K.N_CODES + codes
href.view(-1).index_add_(0, flat.reshape(-1), torch.ones_like(flat.reshape(-1)))
d = (hist - href)
res["kernel_hist_abs_diff"] = int(d.abs().sum())
res["kernel_hist_disp"] = int(d.cumsum(-1).abs().sum())
res["torch"] = torch.__version__
print(json.dumps(res))
