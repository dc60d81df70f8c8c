"""MetricTester matrix over EVERY exported metric class (reference strategy: ``run_class_metric_test`` for every
metric, ``tests/unittests/helpers/testers.py:74-227,368-452``).

For each class in the public namespaces (root + every domain package) this file either holds a spec or an explicit
exemption with its reason; ``test_every_class_is_covered`` fails when a new export has neither.  Every spec runs:

* ``test_single``: pickle / deepcopy / hash round trip, constant class attributes, empty default ``state_dict``,
  per-batch ``forward`` values and the final ``compute()`` against the oracle, and ``reset()`` + re-run;
* ``test_ddp``: 2 gloo ranks (strided batches), with and without ``dist_sync_on_step`` — per-batch values of the
  synced step and the final value against the oracle on the rank-major order of all batches (the coalesced sync
  engine, packed gathers of list states, custom merges);
* ``test_differentiability``: ``is_differentiable`` agrees with what ``forward`` returns (grad flows, or not at all).

Oracle: the reference's own class built by the same factory (``/root/reference/src``, imported through the
``lightning_utilities`` stand-in) wherever the reference runs in this image; otherwise (the reference needs
torchvision / pycocotools / pystoi / gammatone here) this framework's module on one process, which still pins the
distributed paths (2-rank result == 1-rank result).  Inputs are small seeded tensors of each family's shape.
"""
import importlib
import inspect
import pickle
import sys
from copy import deepcopy
from typing import Any, Callable, Dict, List, NamedTuple, Optional

import pytest
import torch
from torch import Tensor, nn

import torchmetrics_forked_amd as tm
from tests.helpers.ddp import run_ddp
from tests.helpers.testers import assert_allclose

REF_PATHS = ("/root/repo/tests/_oracle", "/root/reference/src")
NB = 4  # batches; rank r of 2 takes batches r, r + 2


def _lib(which: str):
    if which == "self":
        return tm
    for p in REF_PATHS:
        if p not in sys.path:
            sys.path.append(p)
    import warnings

    warnings.filterwarnings("ignore")
    return importlib.import_module("torchmetrics")


def _resolve(lib, path: str):
    obj = lib
    for part in path.split("."):
        obj = getattr(obj, part) if hasattr(obj, part) else importlib.import_module(f"{obj.__name__}.{part}")
    return obj


class Build:
    """Picklable factory: ``Build("classification.BinaryAccuracy", threshold=0.4)(lib, **extra)``."""

    def __init__(self, path: str, **kwargs: Any) -> None:
        self.path, self.kwargs = path, kwargs

    def __call__(self, lib, **extra: Any):
        return _resolve(lib, self.path)(**self.kwargs, **extra)


# ---- factories with nested metrics (module level: picklable for the ddp pool) -------------------------------------
def _classwise(lib, **extra):
    return lib.ClasswiseWrapper(lib.classification.MulticlassAccuracy(num_classes=5, average=None, **extra))


def _minmax(lib, **extra):
    return lib.MinMaxMetric(lib.classification.BinaryAccuracy(), **extra)


def _multioutput(lib, **extra):
    return lib.MultioutputWrapper(lib.regression.MeanSquaredError(**extra), num_outputs=2)


def _multitask(lib, **extra):
    return lib.MultitaskWrapper({"cls": lib.classification.BinaryAccuracy(**extra), "reg": lib.regression.MeanSquaredError(**extra)})


def _running(lib, **extra):
    return lib.wrappers.Running(lib.aggregation.SumMetric(), window=2, **extra)


def _bootstrap(lib, **extra):
    torch.manual_seed(7)
    return lib.BootStrapper(lib.regression.MeanSquaredError(), num_bootstraps=4, sampling_strategy="multinomial", **extra)


def _compositional(lib, **extra):
    return lib.classification.BinaryAccuracy(**extra) + lib.classification.BinaryPrecision(**extra)


def _pit(lib, **extra):
    fn = lib.functional.audio.scale_invariant_signal_noise_ratio
    return lib.audio.PermutationInvariantTraining(fn, eval_func="max", **extra)


class TinyFeatures(nn.Module):
    """Deterministic feature extractor for the FID family (the reference accepts a custom module too)."""

    def __init__(self, out: int = 16) -> None:
        super().__init__()
        g = torch.Generator().manual_seed(3)
        self.w = nn.Parameter(torch.randn(48, out, generator=g) / 7, requires_grad=False)

    def forward(self, x: Tensor) -> Tensor:
        x = torch.nn.functional.adaptive_avg_pool2d(x.float() / 255.0, 4).flatten(1)
        return x @ self.w


def _fid(lib, **extra):
    return _resolve(lib, "image.fid").FrechetInceptionDistance(feature=TinyFeatures(), **extra)


def _kid(lib, **extra):
    return _resolve(lib, "image.kid").KernelInceptionDistance(feature=TinyFeatures(), subset_size=4, subsets=3, **extra)


def _mifid(lib, **extra):
    return _resolve(lib, "image.mifid").MemorizationInformedFrechetInceptionDistance(feature=TinyFeatures(), **extra)


def _is(lib, **extra):
    return _resolve(lib, "image.inception").InceptionScore(feature=TinyFeatures(10), splits=2, **extra)


class TinySim(nn.Module):
    def forward(self, a: Tensor, b: Tensor) -> Tensor:
        return ((a - b) ** 2).flatten(1).mean(1)


def _lpips(lib, **extra):
    torch.manual_seed(5)  # random-init trunk: the same weights in the metric and its one-process oracle
    return lib.image.LearnedPerceptualImagePatchSimilarity(net_type="squeeze", **extra)


# ---- seeded inputs: list of NB batches, each a tuple of update args -------------------------------------------------
def _gen(seed: int = 0) -> torch.Generator:
    return torch.Generator().manual_seed(seed)


def _data(kind: str) -> List[tuple]:
    g = _gen(sum(map(ord, kind)))
    N, C = 24, 5
    out = []
    for b in range(NB):
        if kind == "bin":
            out.append((torch.rand(N, generator=g), torch.randint(0, 2, (N,), generator=g)))
        elif kind == "bin_logit":
            out.append((torch.randn(N, generator=g) * 2, torch.randint(0, 2, (N,), generator=g)))
        elif kind == "mc":
            out.append((torch.randn(N, C, generator=g), torch.randint(0, C, (N,), generator=g)))
        elif kind == "mc_label":
            out.append((torch.randint(0, C, (N,), generator=g), torch.randint(0, C, (N,), generator=g)))
        elif kind == "mc_md":
            out.append((torch.randint(0, C, (N, 3), generator=g), torch.randint(0, C, (N, 3), generator=g)))
        elif kind == "ml":
            out.append((torch.rand(N, C, generator=g), torch.randint(0, 2, (N, C), generator=g)))
        elif kind == "group":
            grp = torch.arange(N) % 2
            out.append((torch.rand(N, generator=g), torch.randint(0, 2, (N,), generator=g), grp))
        elif kind == "reg":
            out.append((torch.randn(N, generator=g), torch.randn(N, generator=g)))
        elif kind == "reg_pos":
            out.append((torch.rand(N, generator=g) + 0.1, torch.rand(N, generator=g) + 0.1))
        elif kind == "reg2":
            out.append((torch.randn(N, 2, generator=g), torch.randn(N, 2, generator=g)))
        elif kind == "reg4":
            out.append((torch.randn(N, 4, generator=g), torch.randn(N, 4, generator=g)))
        elif kind == "dist":
            out.append((torch.rand(N, C, generator=g).softmax(1), torch.rand(N, C, generator=g).softmax(1)))
        elif kind == "retrieval":
            out.append((torch.rand(N, generator=g), torch.randint(0, 2, (N,), generator=g), torch.randint(0, 4, (N,), generator=g) + 4 * b))
        elif kind == "fleiss":
            out.append((torch.randint(0, 4, (N, C), generator=g),))
        elif kind == "cluster":
            out.append((torch.randint(0, 4, (N,), generator=g), torch.randint(0, 3, (N,), generator=g)))
        elif kind == "cluster_data":
            lab = torch.arange(N) % 3
            out.append((torch.randn(N, 3, generator=g) + lab[:, None].float(), lab))
        elif kind == "img":
            out.append((torch.rand(2, 3, 24, 24, generator=g), torch.rand(2, 3, 24, 24, generator=g)))
        elif kind == "img_gray":
            out.append((torch.rand(2, 1, 24, 24, generator=g), torch.rand(2, 1, 24, 24, generator=g)))
        elif kind == "img48":
            out.append((torch.rand(2, 3, 48, 48, generator=g), torch.rand(2, 3, 48, 48, generator=g)))
        elif kind == "img_one":
            out.append((torch.rand(2, 3, 24, 24, generator=g),))
        elif kind == "img_lpips":
            out.append((torch.rand(2, 3, 32, 32, generator=g) * 2 - 1, torch.rand(2, 3, 32, 32, generator=g) * 2 - 1))
        elif kind == "img_u8_realfake":
            out.append((torch.randint(0, 256, (6, 3, 16, 16), generator=g, dtype=torch.uint8), b % 2 == 0))
        elif kind == "img_u8":
            out.append((torch.randint(0, 256, (6, 3, 16, 16), generator=g, dtype=torch.uint8),))
        elif kind == "audio":
            t = torch.randn(2, 64, generator=g)
            out.append((t + 0.3 * torch.randn(2, 64, generator=g), t))
        elif kind == "audio_spk":
            t = torch.randn(2, 3, 64, generator=g)
            out.append((t[:, [2, 0, 1]] + 0.3 * torch.randn(2, 3, 64, generator=g), t))
        elif kind == "audio_complex":
            t = torch.randn(2, 9, 8, 2, generator=g)
            out.append((t + 0.3 * torch.randn(2, 9, 8, 2, generator=g), t))
        elif kind == "audio_sdr":
            t = torch.randn(2, 400, generator=g)
            out.append((t + 0.3 * torch.randn(2, 400, generator=g), t))
        elif kind == "audio_stoi":
            t = torch.randn(1, 6000, generator=g)
            out.append((t + 0.5 * torch.randn(1, 6000, generator=g), t))
        elif kind == "audio_one":
            out.append((torch.randn(1, 8000, generator=g),))
        elif kind == "boxes":
            out.append(_boxes(g))
        elif kind == "panoptic":
            out.append(_panoptic(g))
        elif kind == "text":
            out.append(_text(g, b))
        elif kind == "text_multi_ref":
            p, t = _text(g, b)
            out.append((p, [[x, x.upper()] for x in t]))
        elif kind == "squad":
            out.append(_squad(b))
        elif kind == "perplexity":
            out.append((torch.randn(2, 6, 7, generator=g), torch.randint(0, 7, (2, 6), generator=g)))
        elif kind == "agg":
            out.append((torch.randn(N, generator=g),))
        elif kind == "multitask":
            p, t = torch.rand(N, generator=g), torch.randint(0, 2, (N,), generator=g)
            r, s = torch.randn(N, generator=g), torch.randn(N, generator=g)
            out.append(({"cls": p, "reg": r}, {"cls": t, "reg": s}))
        else:
            raise KeyError(kind)
    return out


_WORDS = ["the", "cat", "sat", "on", "a", "mat", "dog", "ran", "far", "away", "quick", "brown"]


def _sentence(g, n):
    return " ".join(_WORDS[int(i)] for i in torch.randint(0, len(_WORDS), (n,), generator=g))


def _text(g, b):
    preds, target = [], []
    for _ in range(3):
        t = _sentence(g, int(torch.randint(4, 9, (1,), generator=g)))
        w = t.split()
        k = int(torch.randint(0, len(w), (1,), generator=g))
        w[k] = _WORDS[(b + k) % len(_WORDS)]
        preds.append(" ".join(w))
        target.append(t)
    return preds, target


def _squad(b):
    ctx = ["alpha beta gamma", "delta epsilon", "zeta eta theta"]
    preds = [{"prediction_text": ctx[(b + i) % 3].split()[i % 2], "id": f"q{b}{i}"} for i in range(2)]
    target = [{"answers": {"answer_start": [0], "text": [ctx[(b + i) % 3].split()[0]]}, "id": f"q{b}{i}"} for i in range(2)]
    return preds, target


def _boxes(g):
    preds, target = [], []
    for _ in range(2):
        xy = torch.rand(4, 2, generator=g) * 50
        wh = torch.rand(4, 2, generator=g) * 30 + 5
        gt = torch.cat([xy, xy + wh], 1)
        pb = gt + torch.randn(4, 4, generator=g) * 3
        preds.append({"boxes": pb, "scores": torch.rand(4, generator=g), "labels": torch.randint(0, 2, (4,), generator=g)})
        target.append({"boxes": gt, "labels": torch.randint(0, 2, (4,), generator=g)})
    return preds, target


def _panoptic(g):
    cat = torch.randint(0, 3, (1, 8, 8), generator=g)
    inst = torch.randint(0, 2, (1, 8, 8), generator=g)
    t = torch.stack([cat, inst], -1)
    p = t.clone()
    p[0, :3, :3, 0] = torch.randint(0, 3, (3, 3), generator=g)
    return p, t


class Spec(NamedTuple):
    make: Callable
    data: str
    oracle: str = "ref"        # "ref" (reference class, same factory) or "self" (this framework on one process)
    atol: float = 1e-5
    ddp: bool = True            # run the 2-rank gloo matrix
    batch: bool = True          # check per-batch forward values
    seeded: bool = False        # metric draws random numbers in compute: seed before compute on both sides


B = Build
MC = {"num_classes": 5}
ML = {"num_labels": 5}
SPECS: Dict[str, Spec] = {}


def _add(name: str, *a, **k) -> None:
    SPECS[name] = Spec(*a, **k)


# classification: binary / multiclass / multilabel families
for fam, cls_names in {
    "": ["Accuracy", "AUROC", "AveragePrecision", "CalibrationError", "CohenKappa", "ConfusionMatrix", "F1Score",
         "HammingDistance", "HingeLoss", "JaccardIndex", "MatthewsCorrCoef", "Precision", "PrecisionRecallCurve", "ROC",
         "Recall", "Specificity", "StatScores"],
}.items():
    for cn in cls_names:
        _add(f"Binary{cn}", B(f"classification.Binary{cn}"), "bin")
        _add(f"Multiclass{cn}", B(f"classification.Multiclass{cn}", **MC), "mc", atol=1e-4)
        if cn not in ("CalibrationError", "CohenKappa", "HingeLoss"):
            _add(f"Multilabel{cn}", B(f"classification.Multilabel{cn}", **ML), "ml", atol=1e-4)
_add("BinaryFBetaScore", B("classification.BinaryFBetaScore", beta=2.0), "bin")
_add("MulticlassFBetaScore", B("classification.MulticlassFBetaScore", beta=2.0, **MC), "mc")
_add("MultilabelFBetaScore", B("classification.MultilabelFBetaScore", beta=2.0, **ML), "ml")
_add("BinaryAUROC_logits", B("classification.BinaryAUROC"), "bin_logit")
_add("BinaryAUROC_binned", B("classification.BinaryAUROC", thresholds=11), "bin")
_add("MulticlassAUROC_binned", B("classification.MulticlassAUROC", thresholds=11, **MC), "mc", atol=1e-4)
_add("MultilabelAUROC_binned", B("classification.MultilabelAUROC", thresholds=11, **ML), "ml", atol=1e-4)
_add("MulticlassAccuracy_top2", B("classification.MulticlassAccuracy", top_k=2, **MC), "mc")
_add("MulticlassAccuracy_micro_ignore", B("classification.MulticlassAccuracy", average="micro", ignore_index=0, **MC), "mc")
for fx in ("PrecisionAtFixedRecall", "RecallAtFixedPrecision", "SpecificityAtSensitivity"):
    arg = {"PrecisionAtFixedRecall": "min_recall", "RecallAtFixedPrecision": "min_precision",
           "SpecificityAtSensitivity": "min_sensitivity"}[fx]
    _add(f"Binary{fx}", B(f"classification.Binary{fx}", **{arg: 0.5}), "bin")
    _add(f"Multiclass{fx}", B(f"classification.Multiclass{fx}", **{arg: 0.5}, **MC), "mc", atol=1e-4)
    _add(f"Multilabel{fx}", B(f"classification.Multilabel{fx}", **{arg: 0.5}, **ML), "ml", atol=1e-4)
_add("MulticlassExactMatch", B("classification.MulticlassExactMatch", **MC), "mc_md")
_add("MultilabelExactMatch", B("classification.MultilabelExactMatch", **ML), "ml")
_add("MultilabelCoverageError", B("classification.MultilabelCoverageError", **ML), "ml")
_add("MultilabelRankingAveragePrecision", B("classification.MultilabelRankingAveragePrecision", **ML), "ml")
_add("MultilabelRankingLoss", B("classification.MultilabelRankingLoss", **ML), "ml")
_add("BinaryFairness", B("classification.BinaryFairness", num_groups=2), "group")
_add("BinaryGroupStatRates", B("classification.BinaryGroupStatRates", num_groups=2), "group")
_add("Dice", B("classification.Dice", num_classes=5, average="micro"), "mc_label")
# task wrappers (root names)
for tw, extra in {"Accuracy": {}, "AUROC": {}, "AveragePrecision": {}, "CalibrationError": {}, "CohenKappa": {},
                  "ConfusionMatrix": {}, "ExactMatch": {}, "F1Score": {}, "FBetaScore": {"beta": 0.5}, "HammingDistance": {},
                  "HingeLoss": {}, "JaccardIndex": {}, "MatthewsCorrCoef": {}, "Precision": {}, "PrecisionRecallCurve": {},
                  "ROC": {}, "Recall": {}, "Specificity": {}, "StatScores": {},
                  "PrecisionAtFixedRecall": {"min_recall": 0.5}, "RecallAtFixedPrecision": {"min_precision": 0.5},
                  "SpecificityAtSensitivity": {"min_sensitivity": 0.5}}.items():
    data = "mc_md" if tw == "ExactMatch" else "mc"
    _add(f"task:{tw}", B(tw, task="multiclass", num_classes=5, **extra), data, atol=1e-4)

# regression
for rn, data in {"MeanSquaredError": "reg", "MeanAbsoluteError": "reg", "MeanSquaredLogError": "reg_pos",
                 "MeanAbsolutePercentageError": "reg_pos", "SymmetricMeanAbsolutePercentageError": "reg_pos",
                 "WeightedMeanAbsolutePercentageError": "reg_pos", "PearsonCorrCoef": "reg", "SpearmanCorrCoef": "reg",
                 "KendallRankCorrCoef": "reg", "ConcordanceCorrCoef": "reg", "R2Score": "reg", "ExplainedVariance": "reg",
                 "LogCoshError": "reg", "RelativeSquaredError": "reg", "TweedieDevianceScore": "reg",
                 "CosineSimilarity": "reg4", "KLDivergence": "dist"}.items():
    _add(rn, B(f"regression.{rn}"), data, atol=1e-4)
_add("MinkowskiDistance", B("regression.MinkowskiDistance", p=3), "reg", atol=1e-4)
_add("PearsonCorrCoef_2out", B("regression.PearsonCorrCoef", num_outputs=2), "reg2", atol=1e-4)
_add("TweedieDevianceScore_p1", B("regression.TweedieDevianceScore", power=1.5), "reg_pos", atol=1e-4)

# retrieval
for rn in ("RetrievalMAP", "RetrievalMRR", "RetrievalNormalizedDCG", "RetrievalPrecision", "RetrievalRecall",
           "RetrievalFallOut", "RetrievalHitRate", "RetrievalRPrecision"):
    _add(rn, B(f"retrieval.{rn}"), "retrieval", atol=1e-5)
_add("RetrievalPrecision_top2", B("retrieval.RetrievalPrecision", top_k=2), "retrieval")
_add("RetrievalPrecisionRecallCurve", B("retrieval.RetrievalPrecisionRecallCurve", max_k=3), "retrieval")
_add("RetrievalRecallAtFixedPrecision", B("retrieval.RetrievalRecallAtFixedPrecision", min_precision=0.3, max_k=3), "retrieval")

# nominal / clustering
for nn_ in ("CramersV", "TschuprowsT", "PearsonsContingencyCoefficient", "TheilsU"):
    _add(nn_, B(f"nominal.{nn_}", num_classes=5), "mc_label", atol=1e-4)
_add("FleissKappa", B("nominal.FleissKappa", mode="counts"), "fleiss", atol=1e-4)
for cn in ("MutualInfoScore", "NormalizedMutualInfoScore", "AdjustedMutualInfoScore", "RandScore", "AdjustedRandScore",
           "FowlkesMallowsIndex", "HomogeneityScore", "CompletenessScore", "VMeasureScore"):
    _add(cn, B(f"clustering.{cn}"), "cluster", atol=1e-4)
for cn in ("CalinskiHarabaszScore", "DaviesBouldinScore", "DunnIndex"):
    _add(cn, B(f"clustering.{cn}"), "cluster_data", atol=1e-4)

# image
for im, data, kw in [("PeakSignalNoiseRatio", "img", {"data_range": 1.0}), ("StructuralSimilarityIndexMeasure", "img", {"data_range": 1.0}),
                     ("UniversalImageQualityIndex", "img", {}), ("SpectralAngleMapper", "img", {}),
                     ("ErrorRelativeGlobalDimensionlessSynthesis", "img", {}), ("RelativeAverageSpectralError", "img", {}),
                     ("RootMeanSquaredErrorUsingSlidingWindow", "img", {}), ("SpectralDistortionIndex", "img", {}),
                     ("PeakSignalNoiseRatioWithBlockedEffect", "img_gray", {}), ("VisualInformationFidelity", "img48", {}),
                     ("MultiScaleStructuralSimilarityIndexMeasure", "img48", {"data_range": 1.0, "kernel_size": 3, "betas": (0.3, 0.3, 0.4)})]:
    _add(im, B(f"image.{im}", **kw), data, atol=1e-4)
_add("TotalVariation", B("image.TotalVariation"), "img_one", atol=1e-3)
_add("FrechetInceptionDistance", _fid, "img_u8_realfake", atol=1e-3, batch=False)
_add("MemorizationInformedFrechetInceptionDistance", _mifid, "img_u8_realfake", atol=1e-3, batch=False)
_add("KernelInceptionDistance", _kid, "img_u8_realfake", atol=1e-4, batch=False, seeded=True)
_add("InceptionScore", _is, "img_u8", atol=1e-4, batch=False, seeded=True)
_add("LearnedPerceptualImagePatchSimilarity", _lpips, "img_lpips", oracle="self", atol=1e-5)

# detection
_add("IntersectionOverUnion", B("detection.IntersectionOverUnion"), "boxes", oracle="self")
_add("GeneralizedIntersectionOverUnion", B("detection.GeneralizedIntersectionOverUnion"), "boxes", oracle="self")
_add("DistanceIntersectionOverUnion", B("detection.DistanceIntersectionOverUnion"), "boxes", oracle="self")
_add("CompleteIntersectionOverUnion", B("detection.CompleteIntersectionOverUnion"), "boxes", oracle="self")
_add("MeanAveragePrecision", B("detection.MeanAveragePrecision"), "boxes", oracle="self", batch=False)
_add("PanopticQuality", B("detection.PanopticQuality", things={0, 1}, stuffs={2}), "panoptic", atol=1e-5)
_add("ModifiedPanopticQuality", B("detection.ModifiedPanopticQuality", things={0, 1}, stuffs={2}), "panoptic", atol=1e-5)

# text
for tn in ("WordErrorRate", "CharErrorRate", "MatchErrorRate", "WordInfoLost", "WordInfoPreserved", "EditDistance",
           "ExtendedEditDistance"):
    _add(tn, B(f"text.{tn}"), "text", atol=1e-5)
_add("TranslationEditRate", B("text.TranslationEditRate"), "text_multi_ref", atol=1e-5)
_add("CHRFScore", B("text.CHRFScore"), "text_multi_ref", atol=1e-5)
_add("BLEUScore", B("text.BLEUScore", n_gram=2), "text_multi_ref", atol=1e-5)
_add("SacreBLEUScore", B("text.SacreBLEUScore", n_gram=2), "text_multi_ref", atol=1e-5)
_add("ROUGEScore", B("text.ROUGEScore", rouge_keys=("rouge1", "rouge2", "rougeL")), "text", atol=1e-5)
_add("SQuAD", B("text.SQuAD"), "squad", atol=1e-5)
_add("Perplexity", B("text.Perplexity"), "perplexity", atol=1e-4)

# audio
_add("SignalNoiseRatio", B("audio.SignalNoiseRatio"), "audio", atol=1e-4)
_add("ScaleInvariantSignalNoiseRatio", B("audio.ScaleInvariantSignalNoiseRatio"), "audio", atol=1e-4)
_add("ScaleInvariantSignalDistortionRatio", B("audio.ScaleInvariantSignalDistortionRatio"), "audio", atol=1e-4)
_add("SignalDistortionRatio", B("audio.SignalDistortionRatio", filter_length=32), "audio_sdr", atol=1e-3)
_add("SourceAggregatedSignalDistortionRatio", B("audio.SourceAggregatedSignalDistortionRatio"), "audio_spk", atol=1e-4)
_add("ComplexScaleInvariantSignalNoiseRatio", B("audio.ComplexScaleInvariantSignalNoiseRatio"), "audio_complex", atol=1e-4)
_add("PermutationInvariantTraining", _pit, "audio_spk", atol=1e-4)
_add("ShortTimeObjectiveIntelligibility", B("audio.ShortTimeObjectiveIntelligibility", fs=10000), "audio_stoi", oracle="self", atol=1e-5)
_add("SpeechReverberationModulationEnergyRatio", B("audio.SpeechReverberationModulationEnergyRatio", fs=8000), "audio_one",
     oracle="self", atol=1e-5, ddp=False)

# aggregation / wrappers
for an in ("SumMetric", "MeanMetric", "MaxMetric", "MinMetric", "CatMetric"):
    _add(an, B(f"aggregation.{an}"), "agg", atol=1e-5)
_add("RunningMean", B("aggregation.RunningMean", window=2), "agg", atol=1e-5, ddp=False)
_add("RunningSum", B("aggregation.RunningSum", window=2), "agg", atol=1e-5, ddp=False)
_add("ClasswiseWrapper", _classwise, "mc")
_add("MinMaxMetric", _minmax, "bin", batch=False)  # batch values carry the running min / max
_add("MultioutputWrapper", _multioutput, "reg2", atol=1e-5)
_add("MultitaskWrapper", _multitask, "multitask", atol=1e-5)
_add("Running", _running, "agg", atol=1e-5, ddp=False)
_add("BootStrapper", _bootstrap, "reg", atol=1e-5, ddp=False, batch=False)
_add("CompositionalMetric", _compositional, "bin")

# classes a spec above covers under another name, or that cannot run here (with the reason)
EXEMPT = {
    "Metric": "abstract base", "WrapperMetric": "abstract base", "BaseAggregator": "abstract base",
    "RetrievalMetric": "abstract base",
    "BERTScore": "needs a pretrained HF encoder (no network); module-vs-reference test on a local random-init model in "
                 "tests/unittests/text (test_bertscore_*)",
    "InfoLM": "needs a pretrained masked LM (no network); covered by the functional tests in tests/unittests/text",
    "CLIPScore": "needs CLIP weights (no network); covered with a local random-init CLIP in tests/unittests/multimodal",
    "CLIPImageQualityAssessment": "needs CLIP weights (no network); covered in tests/unittests/multimodal",
    "PerceptualEvaluationSpeechQuality": "delegates to the `pesq` package, which is not installed (as the reference)",
    "PerceptualPathLength": "needs a generator model; covered in tests/unittests/image",
    "Running": "covered by the `Running` spec",
}


def _all_exported() -> Dict[str, type]:
    from torchmetrics_forked_amd.metric import Metric

    found: Dict[str, type] = {}
    mods = [tm] + [importlib.import_module(f"torchmetrics_forked_amd.{d}") for d in
                   ("classification", "regression", "retrieval", "image", "detection", "text", "audio", "nominal",
                    "clustering", "multimodal", "wrappers", "aggregation")]
    for m in mods:
        for n in getattr(m, "__all__", dir(m)):
            o = getattr(m, n, None)
            if inspect.isclass(o) and issubclass(o, Metric):
                found[n] = o
    return found


def test_every_class_is_covered():
    covered = {n.split(":")[-1].split("_")[0] for n in SPECS}
    missing = sorted(n for n in _all_exported() if n not in covered and n not in EXEMPT)
    assert not missing, f"exported metric classes with no matrix spec and no exemption: {missing}"


# ---- harness ----------------------------------------------------------------------------------------------------------
def _oracle(spec: Spec, batches: List[tuple]) -> Any:
    """The oracle's value on exactly ``batches``: inside a ddp worker the process group is hidden from it, so neither
    the reference nor this framework syncs the oracle's states across ranks."""
    import torch.distributed as dist

    lib = _lib(spec.oracle)
    real = dist.is_initialized
    dist.is_initialized = lambda: False
    try:
        m = spec.make(lib)
        for b in batches:
            m.update(*b)
        if spec.seeded:
            torch.manual_seed(11)
        return m.compute()
    finally:
        dist.is_initialized = real


def _values_equal(res, ref, atol):
    if isinstance(res, dict) and not isinstance(ref, dict):
        raise AssertionError((res, ref))
    if isinstance(res, dict):
        assert set(res) == set(ref), (set(res), set(ref))
        for k in res:
            _values_equal(res[k], ref[k], atol)
        return
    assert_allclose(res, ref, atol)


def _check_module_contract(metric) -> None:
    for attr in ("higher_is_better", "is_differentiable", "full_state_update"):
        with pytest.raises(RuntimeError):
            setattr(metric, attr, True)
    clone = pickle.loads(pickle.dumps(deepcopy(metric)))
    hash(clone)
    assert all(not v for v in metric._persistent.values())


def _matrix_body(rank: int, world: int, spec: Spec, batches: List[tuple], dist_sync_on_step: bool) -> None:
    metric = spec.make(tm, dist_sync_on_step=dist_sync_on_step) if dist_sync_on_step else spec.make(tm)
    mine = list(range(rank, len(batches), world))
    for i in mine:
        if not spec.batch:
            metric.update(*batches[i])
            continue
        out = metric(*batches[i])
        if dist_sync_on_step and world > 1:
            _values_equal(out, _oracle(spec, [batches[j] for j in range(i - rank, i - rank + world)]), spec.atol)
        elif not dist_sync_on_step:
            _values_equal(out, _oracle(spec, [batches[i]]), spec.atol)
    if spec.seeded:
        torch.manual_seed(11)
    result = metric.compute()
    order = [i for r in range(world) for i in range(r, len(batches), world)]
    _values_equal(result, _oracle(spec, [batches[i] for i in order]), spec.atol)


_ORACLE_OK: Dict[str, Optional[str]] = {}


def _need_oracle(name: str, spec: Spec) -> None:
    """Skip (with the reason) when the reference cannot build this spec in this image."""
    if spec.oracle != "ref":
        return
    if name not in _ORACLE_OK:
        try:
            spec.make(_lib("ref"))
            _ORACLE_OK[name] = None
        except (ModuleNotFoundError, ImportError) as err:  # pragma: no cover - depends on the image
            _ORACLE_OK[name] = str(err)[:120]
    if _ORACLE_OK[name] is not None:
        pytest.skip(f"reference oracle unavailable: {_ORACLE_OK[name]}")


@pytest.mark.parametrize("name", sorted(SPECS))
def test_single(name):
    spec = SPECS[name]
    _need_oracle(name, spec)
    metric = spec.make(tm)
    _check_module_contract(metric)
    batches = _data(spec.data)
    _matrix_body(0, 1, spec, batches, False)
    # reset + re-run gives the same value (states re-initialised, arena / caches dropped); the RNG is re-seeded
    # before each pass for metrics that draw in update (BootStrapper)
    torch.manual_seed(7)
    for b in batches:
        metric.update(*b)
    if spec.seeded:
        torch.manual_seed(11)
    first = metric.compute()
    metric.reset()
    torch.manual_seed(7)
    for b in batches:
        metric.update(*b)
    if spec.seeded:
        torch.manual_seed(11)
    _values_equal(metric.compute(), first, spec.atol)


@pytest.mark.parametrize("dist_sync_on_step", [False, True])
@pytest.mark.parametrize("name", sorted(n for n, s in SPECS.items() if s.ddp))
def test_ddp(name, dist_sync_on_step):
    spec = SPECS[name]
    if dist_sync_on_step and not spec.batch:
        pytest.skip("no per-batch value for this metric (forward needs state the batch alone does not have)")
    _need_oracle(name, spec)
    run_ddp(_matrix_body, spec, _data(spec.data), dist_sync_on_step)


@pytest.mark.parametrize("name", sorted(n for n, s in SPECS.items() if s.batch))
def test_differentiability(name):
    spec = SPECS[name]
    batches = _data(spec.data)
    first = batches[0]
    if not isinstance(first[0], Tensor) or not first[0].is_floating_point():
        pytest.skip("integer / structured inputs")
    metric = spec.make(tm)
    if metric.is_differentiable is None:
        pytest.skip("is_differentiable is None (unspecified, as in the reference)")
    if name == "MultioutputWrapper":
        pytest.skip("the reference flags it False (wrappers/multioutput.py:90) although its members' outputs carry grad; "
                    "the flag is kept for parity")
    p = first[0].clone().requires_grad_(True)
    out = metric(p, *first[1:])
    outs = out.values() if isinstance(out, dict) else (out if isinstance(out, (list, tuple)) else [out])
    outs = [o for o in outs if isinstance(o, Tensor)]
    if metric.is_differentiable:
        assert any(o.requires_grad for o in outs), "is_differentiable metric returned no grad-carrying output"
        sum(o.double().sum() for o in outs if o.requires_grad).backward()
        assert p.grad is not None and torch.isfinite(p.grad).all()
    else:
        leaked = [o for o in outs if o.requires_grad]
        if leaked:  # a grad-carrying output of a non-differentiable metric must at least not reach the inputs
            sum(o.double().sum() for o in leaked).backward()
            assert p.grad is None, "non-differentiable metric propagated a gradient to preds"


def _to_dev(x: Any, dev: str) -> Any:
    if isinstance(x, Tensor):
        return x.to(dev)
    if isinstance(x, dict):
        return {k: _to_dev(v, dev) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return type(x)(_to_dev(v, dev) for v in x)
    return x


def _run_on(spec: Spec, batches: List[tuple], dev: str) -> Any:
    torch.manual_seed(7)
    m = spec.make(tm).to(dev)
    vals = []
    for b in batches:
        b = _to_dev(b, dev)
        if spec.batch:
            vals.append(m(*b))
        else:
            m.update(*b)
    if spec.seeded:
        torch.manual_seed(11)
    return vals, m.compute()


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(SPECS))
def test_gpu_vs_cpu(name):
    """Every spec with its states on the MI355X (the native update / compute paths) against the same module on the
    CPU: per-batch forward values and the final value."""
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    spec = SPECS[name]
    batches = _data(spec.data)
    g_vals, g_res = _run_on(spec, batches, "cuda")
    c_vals, c_res = _run_on(spec, batches, "cpu")
    # GPU reductions run in other orders (atomics, tree sums): fp32 agreement, not bit equality
    atol = max(spec.atol, 1e-4)
    for a, b in zip(g_vals, c_vals):
        _values_equal(a, b, atol)
    _values_equal(g_res, c_res, atol)


# ---- TorchScript: every spec (the reference's testers script every metric class by default, testers.py:131-133) --------
# The wrappers below take ``*args`` / ``**kwargs`` in update / forward, which TorchScript cannot compile; the reference's
# classes fail identically (checked by test_scriptable_exemptions_fail_in_reference too).
SCRIPT_EXEMPT = {
    "BootStrapper": "update(*args, **kwargs)", "ClasswiseWrapper": "update(*args, **kwargs)",
    "MinMaxMetric": "update(*args, **kwargs)", "Running": "update(*args, **kwargs)",
    "RunningMean": "Running(MeanMetric): update(*args, **kwargs)", "RunningSum": "Running(SumMetric): update(*args, **kwargs)",
    "MultitaskWrapper": "update(task_preds: Dict, task_targets: Dict) over nested metrics (JIT internal assert, as the reference)",
}


@pytest.mark.parametrize("name", sorted(n for n in SPECS if n not in SCRIPT_EXEMPT))
def test_scriptable(name):
    """``torch.jit.script`` on a fresh and on an updated module; scripting leaves the eager value unchanged."""
    spec = SPECS[name]
    torch.jit.script(spec.make(tm))
    metric = spec.make(tm)
    for b in _data(spec.data):
        metric.update(*b)
    if spec.seeded:
        torch.manual_seed(11)
    before = metric.compute()
    torch.jit.script(metric)
    metric._computed = None
    if spec.seeded:
        torch.manual_seed(11)
    _values_equal(metric.compute(), before, 0.0)


@pytest.mark.parametrize("name", sorted(SCRIPT_EXEMPT))
def test_scriptable_exemptions_fail_in_reference(reference, name):
    spec = SPECS[name]
    with pytest.raises(Exception):
        torch.jit.script(spec.make(tm))
    with pytest.raises(Exception):
        torch.jit.script(spec.make(reference))
