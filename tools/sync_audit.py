"""Which metric updates synchronise the host with the GPU?  Runs update() under torch.cuda.set_sync_debug_mode
("warn") and counts the synchronising calls per metric (after a warm-up update)."""
import json
import os
import sys
import warnings

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import torchmetrics_forked_amd as tm  # noqa: E402
from torchmetrics_forked_amd import ops  # noqa: E402

ops.require()
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
N, C = 4096, 10
mc_p = torch.randn(N, C, device=dev, generator=g).softmax(1)
mc_t = torch.randint(0, C, (N,), device=dev, generator=g)
b_p = torch.rand(N, device=dev, generator=g)
b_t = torch.randint(0, 2, (N,), device=dev, generator=g)
ml_p = torch.rand(N, 5, device=dev, generator=g)
ml_t = torch.randint(0, 2, (N, 5), device=dev, generator=g)
r_p = torch.randn(N, device=dev, generator=g)
r_t = torch.randn(N, device=dev, generator=g)
img_p = torch.rand(4, 3, 64, 64, device=dev, generator=g)
img_t = torch.rand(4, 3, 64, 64, device=dev, generator=g)
cases = {
    "BinaryAccuracy": (tm.classification.BinaryAccuracy(), (b_p, b_t)),
    "BinaryAUROC": (tm.classification.BinaryAUROC(), (b_p.bfloat16(), b_t)),
    "BinaryAUROC_binned": (tm.classification.BinaryAUROC(thresholds=50), (b_p, b_t)),
    "BinaryAveragePrecision": (tm.classification.BinaryAveragePrecision(), (b_p.bfloat16(), b_t)),
    "BinaryCalibrationError": (tm.classification.BinaryCalibrationError(), (b_p, b_t)),
    "MulticlassAccuracy": (tm.classification.MulticlassAccuracy(num_classes=C), (mc_p, mc_t)),
    "MulticlassF1Score": (tm.classification.MulticlassF1Score(num_classes=C), (mc_p, mc_t)),
    "MulticlassConfusionMatrix": (tm.classification.MulticlassConfusionMatrix(num_classes=C), (mc_p, mc_t)),
    "MulticlassAUROC": (tm.classification.MulticlassAUROC(num_classes=C), (mc_p.bfloat16(), mc_t)),
    "MulticlassAUROC_binned": (tm.classification.MulticlassAUROC(num_classes=C, thresholds=50), (mc_p, mc_t)),
    "MulticlassCalibrationError": (tm.classification.MulticlassCalibrationError(num_classes=C), (mc_p, mc_t)),
    "MulticlassCohenKappa": (tm.classification.MulticlassCohenKappa(num_classes=C), (mc_p, mc_t)),
    "MulticlassMatthewsCorrCoef": (tm.classification.MulticlassMatthewsCorrCoef(num_classes=C), (mc_p, mc_t)),
    "MulticlassHingeLoss": (tm.classification.MulticlassHingeLoss(num_classes=C), (mc_p, mc_t)),
    "BinaryHingeLoss": (tm.classification.BinaryHingeLoss(), (b_p, mc_t % 2)),
    "MulticlassJaccardIndex": (tm.classification.MulticlassJaccardIndex(num_classes=C), (mc_p, mc_t)),
    "MulticlassExactMatch": (tm.classification.MulticlassExactMatch(num_classes=C), (mc_p.argmax(1).reshape(64, 64), mc_t.reshape(64, 64))),
    "MultilabelAccuracy": (tm.classification.MultilabelAccuracy(num_labels=5), (ml_p, ml_t)),
    "MultilabelAUROC": (tm.classification.MultilabelAUROC(num_labels=5), (ml_p.bfloat16(), ml_t)),
    "MultilabelRankingLoss": (tm.classification.MultilabelRankingLoss(num_labels=5), (ml_p, ml_t)),
    "MeanSquaredError": (tm.regression.MeanSquaredError(), (r_p, r_t)),
    "MeanAbsoluteError": (tm.regression.MeanAbsoluteError(), (r_p, r_t)),
    "R2Score": (tm.regression.R2Score(), (r_p, r_t)),
    "PearsonCorrCoef": (tm.regression.PearsonCorrCoef(), (r_p, r_t)),
    "SpearmanCorrCoef": (tm.regression.SpearmanCorrCoef(), (r_p, r_t)),
    "CosineSimilarity": (tm.regression.CosineSimilarity(), (r_p.reshape(64, 64), r_t.reshape(64, 64))),
    "MeanAbsolutePercentageError": (tm.regression.MeanAbsolutePercentageError(), (r_p, r_t)),
    "KLDivergence": (tm.regression.KLDivergence(), (mc_p, mc_p.flip(1))),
    "MeanMetric": (tm.aggregation.MeanMetric(), (r_p,)),
    "SumMetric": (tm.aggregation.SumMetric(), (r_p,)),
    "MaxMetric": (tm.aggregation.MaxMetric(), (r_p,)),
    "CatMetric": (tm.aggregation.CatMetric(), (r_p,)),
    "PeakSignalNoiseRatio": (tm.image.PeakSignalNoiseRatio(data_range=1.0), (img_p, img_t)),
    "StructuralSimilarityIndexMeasure": (tm.image.StructuralSimilarityIndexMeasure(data_range=1.0), (img_p, img_t)),
    "RetrievalMAP": (tm.retrieval.RetrievalMAP(), (b_p, b_t.bool(), torch.randint(0, 50, (N,), device=dev, generator=g))),
    "RetrievalNormalizedDCG": (tm.retrieval.RetrievalNormalizedDCG(), (b_p, b_t.bool(), torch.randint(0, 50, (N,), device=dev, generator=g))),
}
import traceback  # noqa: E402

where = {}


def first_sync_site(m, args):
    """Re-run with sync debug mode 'error' and return the innermost package frames of the first sync."""
    torch.cuda.set_sync_debug_mode("error")
    try:
        m.update(*args)
    except RuntimeError:
        frames = [f for f in traceback.extract_tb(sys.exc_info()[2]) if "torchmetrics_forked_amd" in f.filename]
        return [f"{os.path.basename(f.filename)}:{f.lineno} {f.line}" for f in frames[-3:]]
    finally:
        torch.cuda.set_sync_debug_mode("default")
    return []


out = {}
# the first update measured under set_sync_debug_mode in a process can report a one-time synchronisation (round 2
# audited BinaryAccuracy at 1 sync with no package frame at the site): measure a throwaway copy of the first case
# before the audited ones, and audit each metric in both orders (first / last) so an order artifact shows up
cases = {"_throwaway": (tm.classification.BinaryAccuracy(), (b_p, b_t)), **cases,
         "BinaryAccuracy_last": (tm.classification.BinaryAccuracy(), (b_p, b_t))}
for name, (m, args) in cases.items():
    m = m.to(dev)
    try:
        m.update(*args)
        m.update(*args)  # two warm-up updates: one-time lazy initialisation is not a per-update sync
        torch.cuda.synchronize()
        with warnings.catch_warnings(record=True) as w:
            warnings.simplefilter("always")
            torch.cuda.set_sync_debug_mode("warn")
            m.update(*args)
            torch.cuda.set_sync_debug_mode("default")
        syncs = [str(x.message).splitlines()[0][:80] for x in w if "synchroniz" in str(x.message).lower()]
        out[name] = len(syncs)
        if syncs:
            where[name] = first_sync_site(m, args) or syncs[:2]
    except Exception as e:  # noqa: BLE001
        torch.cuda.set_sync_debug_mode("default")
        out[name] = f"error: {type(e).__name__}: {str(e)[:80]}"
out.pop("_throwaway", None)
where.pop("_throwaway", None)
print(json.dumps({"syncs_per_update": out, "first_sync_site": where}, indent=1))
