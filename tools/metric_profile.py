"""torch.profiler breakdown (host ops + GPU kernels) of a few metric updates: python tools/metric_profile.py <case>."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import torchmetrics_forked_amd as tm  # noqa: E402
from torchmetrics_forked_amd import ops  # noqa: E402

ops.require()
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
NB = 1 << 24
N, C = 65536, 1000


def make(name):
    if name == "binary_auroc_binned":
        return tm.BinaryAUROC(thresholds=100), (torch.rand(NB, device=dev, generator=g), torch.randint(0, 2, (NB,), device=dev, generator=g))
    if name == "multilabel_auroc":
        return tm.MultilabelAUROC(num_labels=1000), (torch.randn(16384, 1000, device=dev, generator=g).bfloat16(),
                                                     torch.randint(0, 2, (16384, 1000), device=dev, generator=g))
    if name == "mc_calibration":
        return tm.MulticlassCalibrationError(num_classes=C), (torch.randn(N, C, device=dev, generator=g).bfloat16(),
                                                              torch.randint(0, C, (N,), device=dev, generator=g))
    if name == "retrieval_map":
        return tm.RetrievalMAP(), (torch.randn(1 << 20, device=dev, generator=g), torch.rand(1 << 20, device=dev, generator=g) > 0.5,
                                   torch.randint(0, 10000, (1 << 20,), device=dev, generator=g))
    if name in ("mse", "r2", "mae"):
        cls = {"mse": tm.MeanSquaredError, "r2": tm.R2Score, "mae": tm.MeanAbsoluteError}[name]
        return cls(), (torch.randn(NB, device=dev, generator=g), torch.randn(NB, device=dev, generator=g))
    if name == "mc_accuracy_c10":
        return tm.MulticlassAccuracy(num_classes=10), (torch.randn(1 << 20, 10, device=dev, generator=g).bfloat16(),
                                                       torch.randint(0, 10, (1 << 20,), device=dev, generator=g))
    raise SystemExit(f"unknown case {name}")


for name in sys.argv[1:]:
    m, inputs = make(name)
    m = m.to(dev)
    for _ in range(3):
        m.update(*inputs)
    torch.cuda.synchronize()
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]) as prof:
        for _ in range(5):
            m.update(*inputs)
        torch.cuda.synchronize()
    print(f"==== {name} (5 updates)")
    print(prof.key_averages().table(sort_by="self_cuda_time_total", row_limit=14, max_name_column_width=70))
    print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=10, max_name_column_width=70))
