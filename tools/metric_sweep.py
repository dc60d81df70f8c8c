"""Update throughput of common metrics on one MI355X: ms per update and effective GB/s of the inputs."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import torchmetrics_forked_amd as tm  # noqa: E402
from torchmetrics_forked_amd import ops  # noqa: E402

ops.require()
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)


def timed(fn, n=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n


def case(name, metric, *inputs):
    m = metric.to(dev)
    nbytes = sum(x.numel() * x.element_size() for x in inputs)
    t = timed(lambda: m.update(*inputs))
    out[name] = {"ms": round(1e3 * t, 3), "GBps": round(nbytes / t / 1e9, 1)}


out = {}
N, C = 65536, 1000
logits = torch.randn(N, C, device=dev, generator=g).bfloat16()
lab = torch.randint(0, C, (N,), device=dev, generator=g)
case("MulticlassAccuracy_C1000_N65536", tm.MulticlassAccuracy(num_classes=C), logits, lab)
case("MulticlassF1_macro_C1000_N65536", tm.MulticlassF1Score(num_classes=C, average="macro"), logits, lab)
case("MulticlassConfusionMatrix_C1000_N65536", tm.MulticlassConfusionMatrix(num_classes=C), logits, lab)
case("MulticlassAveragePrecision_C1000_N65536", tm.MulticlassAveragePrecision(num_classes=C), logits, lab)
case("MulticlassCalibrationError_C1000_N65536", tm.MulticlassCalibrationError(num_classes=C), logits, lab)
NB = 1 << 24
bp = torch.rand(NB, device=dev, generator=g)
bt = torch.randint(0, 2, (NB,), device=dev, generator=g)
case("BinaryAccuracy_N16M_fp32", tm.BinaryAccuracy(), bp, bt)
case("BinaryF1_N16M_fp32", tm.BinaryF1Score(), bp, bt)
case("BinaryAUROC_N16M_fp32_thresholds100", tm.BinaryAUROC(thresholds=100), bp, bt)
mlp = torch.randn(16384, 1000, device=dev, generator=g).bfloat16()
mlt = torch.randint(0, 2, (16384, 1000), device=dev, generator=g)
case("MultilabelF1_L1000_N16384", tm.MultilabelF1Score(num_labels=1000), mlp, mlt)
case("MultilabelAUROC_L1000_N16384", tm.MultilabelAUROC(num_labels=1000), mlp, mlt)
rp = torch.randn(NB, device=dev, generator=g)
rt = torch.randn(NB, device=dev, generator=g)
case("MeanSquaredError_N16M", tm.MeanSquaredError(), rp, rt)
case("PearsonCorrCoef_N16M", tm.PearsonCorrCoef(), rp, rt)
case("R2Score_N16M", tm.R2Score(), rp, rt)
case("SpearmanCorrCoef_N1M", tm.SpearmanCorrCoef(), rp[: 1 << 20], rt[: 1 << 20])
qi = torch.randint(0, 10000, (1 << 20,), device=dev, generator=g)
case("RetrievalMAP_N1M_Q10k", tm.RetrievalMAP(), rp[: 1 << 20], (rt[: 1 << 20] > 0), qi)
print(json.dumps(out))
