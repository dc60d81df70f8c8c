"""Small-class (C = 10) MulticlassAUROC updates only, 1M bf16 rows (for counter passes of the small-class kernels)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import torchmetrics_forked_amd as tm  # noqa: E402
from torchmetrics_forked_amd import ops  # noqa: E402

ops.require()
dev = torch.device("cuda", 0)
C, N = int(os.environ.get("SMALL_C", "10")), 1 << 20
p = torch.randn(N, C, device=dev).bfloat16()
t = torch.randint(0, C, (N,), device=dev)
m = tm.MulticlassAUROC(num_classes=C).to(dev)
for _ in range(8):
    m.update(p, t)
torch.cuda.synchronize()
print("ok")
