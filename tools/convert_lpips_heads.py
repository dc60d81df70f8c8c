"""Build ``torchmetrics_forked_amd/models/lpips_heads.safetensors`` — the LPIPS linear-head weights (1x1 convs over
each backbone stage, as published by the LPIPS authors) — from the reference's ``lpips_models/{alex,vgg,squeeze}.pth``.

The ``.pth`` files are read with ``torch.load(..., weights_only=True)`` (nothing from them is executed) and only the
``lin{i}.model.1.weight`` tensors are kept, flattened to ``{net}.lin{i}`` float32 vectors in a safetensors file, so
the package loads its default heads without unpickling anything.

Usage: python tools/convert_lpips_heads.py [reference_lpips_models_dir]
"""
import os
import sys

import torch
from safetensors.torch import save_file

SRC = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/src/torchmetrics/functional/image/lpips_models"
DST = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "torchmetrics_forked_amd", "models", "lpips_heads.safetensors")

out = {}
for net in ("alex", "vgg", "squeeze"):
    state = torch.load(os.path.join(SRC, f"{net}.pth"), map_location="cpu", weights_only=True)
    for key, val in state.items():
        layer = key.split(".")[0]  # lin{i}
        out[f"{net}.{layer}"] = val.reshape(-1).to(torch.float32).contiguous()
save_file(out, DST, metadata={"source": "LPIPS v0.1 linear heads (reference lpips_models/*.pth)", "layout": "{net}.lin{i}: [C]"})
print(f"wrote {DST}: {len(out)} tensors, {sum(v.numel() for v in out.values())} weights")
