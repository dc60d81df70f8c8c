"""Insert runnable ``Example:`` sections (doctest format) into public class docstrings.

Each spec is (module file, class name, one-line summary used when the class has no docstring, example lines).  The
lines are executed here, on CPU, and every expression's ``repr`` becomes the expected output, so the examples are
exactly what the library prints.  ``tests/unittests/misc/test_doctests.py`` runs them as doctests.

Usage: python tools/gen_doc_examples.py [--check]   (``--check``: only report classes whose example is missing)
"""
import ast
import io
import os
import sys
from contextlib import redirect_stdout
from typing import List, Tuple

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = os.path.join(ROOT, "torchmetrics_forked_amd")

T = "import torch"
SPECS: List[Tuple[str, str, str, List[str]]] = [
    ("classification/accuracy.py", "BinaryAccuracy", "Accuracy for binary tasks.", [
        T, "from torchmetrics_forked_amd.classification import BinaryAccuracy",
        "metric = BinaryAccuracy()", "metric(torch.tensor([0.1, 0.8, 0.6, 0.3]), torch.tensor([0, 1, 0, 0]))"]),
    ("classification/accuracy.py", "MulticlassAccuracy", "Accuracy for multiclass tasks.", [
        T, "from torchmetrics_forked_amd.classification import MulticlassAccuracy",
        "target = torch.tensor([2, 1, 0, 0])", "preds = torch.tensor([2, 1, 0, 1])",
        "MulticlassAccuracy(num_classes=3)(preds, target)", "MulticlassAccuracy(num_classes=3, average=None)(preds, target)"]),
    ("classification/accuracy.py", "MultilabelAccuracy", "Accuracy for multilabel tasks.", [
        T, "from torchmetrics_forked_amd.classification import MultilabelAccuracy",
        "target = torch.tensor([[0, 1, 0], [1, 0, 1]])", "preds = torch.tensor([[0.2, 0.9, 0.1], [0.7, 0.4, 0.3]])",
        "MultilabelAccuracy(num_labels=3)(preds, target)"]),
    ("classification/f_beta.py", "MulticlassF1Score", "F1 score for multiclass tasks.", [
        T, "from torchmetrics_forked_amd.classification import MulticlassF1Score",
        "metric = MulticlassF1Score(num_classes=3)", "metric(torch.tensor([2, 1, 0, 1]), torch.tensor([2, 1, 0, 0]))"]),
    ("classification/precision_recall.py", "MulticlassPrecision", "Precision for multiclass tasks.", [
        T, "from torchmetrics_forked_amd.classification import MulticlassPrecision",
        "metric = MulticlassPrecision(num_classes=3, average='micro')", "metric(torch.tensor([2, 1, 0, 1]), torch.tensor([2, 1, 0, 0]))"]),
    ("classification/precision_recall.py", "MulticlassRecall", "Recall for multiclass tasks.", [
        T, "from torchmetrics_forked_amd.classification import MulticlassRecall",
        "metric = MulticlassRecall(num_classes=3, average=None)", "metric(torch.tensor([2, 1, 0, 1]), torch.tensor([2, 1, 0, 0]))"]),
    ("classification/auroc.py", "MulticlassAUROC", "One-vs-rest AUROC for multiclass tasks.", [
        T, "from torchmetrics_forked_amd.classification import MulticlassAUROC",
        "preds = torch.tensor([[0.75, 0.05, 0.20], [0.05, 0.75, 0.20], [0.05, 0.05, 0.90], [0.20, 0.10, 0.70]])",
        "target = torch.tensor([0, 1, 2, 2])", "MulticlassAUROC(num_classes=3)(preds, target)",
        "MulticlassAUROC(num_classes=3, average=None)(preds, target)"]),
    ("classification/auroc.py", "BinaryAUROC", "Area under the ROC curve for binary tasks.", [
        T, "from torchmetrics_forked_amd.classification import BinaryAUROC",
        "metric = BinaryAUROC()", "metric(torch.tensor([0.1, 0.4, 0.35, 0.8]), torch.tensor([0, 0, 1, 1]))"]),
    ("classification/average_precision.py", "MulticlassAveragePrecision", "One-vs-rest AveragePrecision for multiclass tasks.", [
        T, "from torchmetrics_forked_amd.classification import MulticlassAveragePrecision",
        "preds = torch.tensor([[0.75, 0.05, 0.20], [0.05, 0.75, 0.20], [0.05, 0.05, 0.90], [0.20, 0.10, 0.70]])",
        "MulticlassAveragePrecision(num_classes=3)(preds, torch.tensor([0, 1, 2, 2]))"]),
    ("classification/confusion_matrix.py", "MulticlassConfusionMatrix", "Confusion matrix for multiclass tasks.", [
        T, "from torchmetrics_forked_amd.classification import MulticlassConfusionMatrix",
        "metric = MulticlassConfusionMatrix(num_classes=3)", "metric(torch.tensor([2, 1, 0, 1]), torch.tensor([2, 1, 0, 0]))"]),
    ("classification/calibration_error.py", "MulticlassCalibrationError", "Top-label calibration error for multiclass tasks.", [
        T, "from torchmetrics_forked_amd.classification import MulticlassCalibrationError",
        "preds = torch.tensor([[0.25, 0.20, 0.55], [0.55, 0.05, 0.40], [0.10, 0.30, 0.60], [0.90, 0.05, 0.05]])",
        "MulticlassCalibrationError(num_classes=3, n_bins=3, norm='l1')(preds, torch.tensor([0, 1, 2, 0]))"]),
    ("classification/cohen_kappa.py", "MulticlassCohenKappa", "Cohen's kappa for multiclass tasks.", [
        T, "from torchmetrics_forked_amd.classification import MulticlassCohenKappa",
        "MulticlassCohenKappa(num_classes=3)(torch.tensor([2, 1, 0, 1]), torch.tensor([2, 1, 0, 0]))"]),
    ("classification/matthews_corrcoef.py", "MulticlassMatthewsCorrCoef", "Matthews correlation coefficient for multiclass tasks.", [
        T, "from torchmetrics_forked_amd.classification import MulticlassMatthewsCorrCoef",
        "MulticlassMatthewsCorrCoef(num_classes=3)(torch.tensor([2, 1, 0, 1]), torch.tensor([2, 1, 0, 0]))"]),
    ("classification/jaccard.py", "MulticlassJaccardIndex", "Jaccard index (IoU) for multiclass tasks.", [
        T, "from torchmetrics_forked_amd.classification import MulticlassJaccardIndex",
        "MulticlassJaccardIndex(num_classes=3)(torch.tensor([2, 1, 0, 1]), torch.tensor([2, 1, 0, 0]))"]),
    ("classification/stat_scores.py", "MulticlassStatScores", "tp / fp / tn / fn / support for multiclass tasks.", [
        T, "from torchmetrics_forked_amd.classification import MulticlassStatScores",
        "metric = MulticlassStatScores(num_classes=3, average=None)", "metric(torch.tensor([2, 1, 0, 1]), torch.tensor([2, 1, 0, 0]))"]),
    ("classification/specificity.py", "MulticlassSpecificity", "Specificity for multiclass tasks.", [
        T, "from torchmetrics_forked_amd.classification import MulticlassSpecificity",
        "MulticlassSpecificity(num_classes=3)(torch.tensor([2, 1, 0, 1]), torch.tensor([2, 1, 0, 0]))"]),
    ("classification/hinge.py", "MulticlassHingeLoss", "Multiclass hinge loss (crammer-singer or one-vs-all).", [
        T, "from torchmetrics_forked_amd.classification import MulticlassHingeLoss",
        "preds = torch.tensor([[0.25, 0.20, 0.55], [0.55, 0.05, 0.40], [0.10, 0.30, 0.60], [0.90, 0.05, 0.05]])",
        "MulticlassHingeLoss(num_classes=3)(preds, torch.tensor([0, 1, 2, 0]))",
        "MulticlassHingeLoss(num_classes=3, multiclass_mode='one-vs-all')(preds, torch.tensor([0, 1, 2, 0]))"]),
    ("classification/ranking.py", "MultilabelRankingLoss", "Label ranking loss for multilabel tasks.", [
        T, "from torchmetrics_forked_amd.classification import MultilabelRankingLoss",
        "preds = torch.tensor([[0.9, 0.2, 0.6], [0.1, 0.8, 0.4], [0.5, 0.3, 0.7]])",
        "MultilabelRankingLoss(num_labels=3)(preds, torch.tensor([[1, 0, 0], [0, 0, 1], [1, 1, 0]]))"]),
    ("classification/exact_match.py", "MulticlassExactMatch", "Exact match (all positions correct) for multiclass tasks.", [
        T, "from torchmetrics_forked_amd.classification import MulticlassExactMatch",
        "target = torch.tensor([[[0, 1], [2, 1], [0, 2]], [[1, 1], [2, 0], [1, 2]]])",
        "preds = torch.tensor([[[0, 1], [2, 1], [0, 2]], [[2, 2], [2, 1], [1, 0]]])",
        "MulticlassExactMatch(num_classes=3, multidim_average='global')(preds, target)"]),
    ("classification/roc.py", "BinaryROC", "ROC curve for binary tasks.", [
        T, "from torchmetrics_forked_amd.classification import BinaryROC",
        "fpr, tpr, thresholds = BinaryROC()(torch.tensor([0.0, 0.5, 0.7, 0.8]), torch.tensor([0, 1, 1, 0]))",
        "fpr", "tpr"]),
    ("classification/precision_recall_curve.py", "BinaryPrecisionRecallCurve", "Precision-recall curve for binary tasks.", [
        T, "from torchmetrics_forked_amd.classification import BinaryPrecisionRecallCurve",
        "precision, recall, thresholds = BinaryPrecisionRecallCurve()(torch.tensor([0.0, 0.5, 0.7, 0.8]), torch.tensor([0, 1, 1, 0]))",
        "precision", "recall"]),
    ("regression/errors.py", "MeanSquaredError", "Mean squared error.", [
        T, "from torchmetrics_forked_amd.regression import MeanSquaredError",
        "MeanSquaredError()(torch.tensor([2.5, 5.0, 4.0, 8.0]), torch.tensor([3.0, 5.0, 2.5, 7.0]))"]),
    ("regression/errors.py", "MeanAbsoluteError", "Mean absolute error.", [
        T, "from torchmetrics_forked_amd.regression import MeanAbsoluteError",
        "MeanAbsoluteError()(torch.tensor([2.5, 0.0, 2.0, 8.0]), torch.tensor([3.0, -0.5, 2.0, 7.0]))"]),
    ("regression/moments.py", "R2Score", "Coefficient of determination.", [
        T, "from torchmetrics_forked_amd.regression import R2Score",
        "R2Score()(torch.tensor([2.5, 0.0, 2.0, 8.0]), torch.tensor([3.0, -0.5, 2.0, 7.0]))"]),
    ("regression/moments.py", "PearsonCorrCoef", "Pearson correlation coefficient.", [
        T, "from torchmetrics_forked_amd.regression import PearsonCorrCoef",
        "PearsonCorrCoef()(torch.tensor([2.5, 0.0, 2.0, 8.0]), torch.tensor([3.0, -0.5, 2.0, 7.0]))"]),
    ("regression/rank.py", "SpearmanCorrCoef", "Spearman rank correlation coefficient.", [
        T, "from torchmetrics_forked_amd.regression import SpearmanCorrCoef",
        "SpearmanCorrCoef()(torch.tensor([2.5, 0.0, 2.0, 8.0]), torch.tensor([3.0, -0.5, 2.0, 7.0]))"]),
    ("regression/kendall.py", "KendallRankCorrCoef", "Kendall rank correlation coefficient (tau-a / b / c).", [
        T, "from torchmetrics_forked_amd.regression import KendallRankCorrCoef",
        "KendallRankCorrCoef()(torch.tensor([2.5, 0.0, 2.0, 8.0]), torch.tensor([3.0, -0.5, 2.0, 7.0]))"]),
    ("regression/moments.py", "ExplainedVariance", "Explained variance.", [
        T, "from torchmetrics_forked_amd.regression import ExplainedVariance",
        "ExplainedVariance()(torch.tensor([2.5, 0.0, 2.0, 8.0]), torch.tensor([3.0, -0.5, 2.0, 7.0]))"]),
    ("retrieval/base.py", "RetrievalMAP", "Mean average precision over queries.", [
        T, "from torchmetrics_forked_amd.retrieval import RetrievalMAP",
        "indexes = torch.tensor([0, 0, 0, 1, 1, 1, 1])", "preds = torch.tensor([0.2, 0.3, 0.5, 0.1, 0.3, 0.5, 0.2])",
        "target = torch.tensor([False, False, True, False, True, False, True])",
        "RetrievalMAP()(preds, target, indexes=indexes)"]),
    ("retrieval/base.py", "RetrievalNormalizedDCG", "Normalized discounted cumulative gain over queries.", [
        T, "from torchmetrics_forked_amd.retrieval import RetrievalNormalizedDCG",
        "indexes = torch.tensor([0, 0, 0, 1, 1, 1, 1])", "preds = torch.tensor([0.2, 0.3, 0.5, 0.1, 0.3, 0.5, 0.2])",
        "target = torch.tensor([0, 0, 2, 0, 1, 0, 3])",
        "RetrievalNormalizedDCG()(preds, target, indexes=indexes)"]),
    ("retrieval/base.py", "RetrievalMRR", "Mean reciprocal rank over queries.", [
        T, "from torchmetrics_forked_amd.retrieval import RetrievalMRR",
        "indexes = torch.tensor([0, 0, 0, 1, 1, 1, 1])", "preds = torch.tensor([0.2, 0.3, 0.5, 0.1, 0.3, 0.5, 0.2])",
        "target = torch.tensor([False, False, True, False, True, False, True])",
        "RetrievalMRR()(preds, target, indexes=indexes)"]),
    ("aggregation.py", "MeanMetric", "Running (weighted) mean.", [
        T, "from torchmetrics_forked_amd.aggregation import MeanMetric",
        "metric = MeanMetric()", "metric.update(1)", "metric.update(torch.tensor([2, 3]))", "metric.compute()"]),
    ("aggregation.py", "SumMetric", "Running sum.", [
        T, "from torchmetrics_forked_amd.aggregation import SumMetric",
        "metric = SumMetric()", "metric.update(1)", "metric.update(torch.tensor([2, 3]))", "metric.compute()"]),
    ("aggregation.py", "MaxMetric", "Running maximum.", [
        T, "from torchmetrics_forked_amd.aggregation import MaxMetric",
        "metric = MaxMetric()", "metric.update(1)", "metric.update(torch.tensor([2, 3]))", "metric.compute()"]),
    ("aggregation.py", "CatMetric", "Concatenation of every value seen.", [
        T, "from torchmetrics_forked_amd.aggregation import CatMetric",
        "metric = CatMetric()", "metric.update(1)", "metric.update(torch.tensor([2, 3]))", "metric.compute()"]),
    ("text/_simple.py", "WordErrorRate", "Word error rate.", [
        "from torchmetrics_forked_amd.text import WordErrorRate",
        "WordErrorRate()(['this is the prediction', 'there is an other sample'], ['this is the reference', 'there is another one'])"]),
    ("text/_simple.py", "CharErrorRate", "Character error rate.", [
        "from torchmetrics_forked_amd.text import CharErrorRate",
        "CharErrorRate()(['this is the prediction', 'there is an other sample'], ['this is the reference', 'there is another one'])"]),
    ("text/_simple.py", "BLEUScore", "BLEU score of a corpus.", [
        "from torchmetrics_forked_amd.text import BLEUScore",
        "BLEUScore()(['the squirrel is eating the nut'], [['a squirrel is eating a nut', 'the squirrel is eating a tasty nut']])"]),
    ("text/_simple.py", "EditDistance", "Levenshtein edit distance.", [
        "from torchmetrics_forked_amd.text import EditDistance",
        "EditDistance()(['rain'], ['shine'])"]),
    ("clustering/_modules.py", "MutualInfoScore", "Mutual information between two clusterings.", [
        T, "from torchmetrics_forked_amd.clustering import MutualInfoScore",
        "MutualInfoScore()(torch.tensor([2, 1, 0, 1, 0]), torch.tensor([0, 2, 1, 1, 0]))"]),
    ("clustering/_modules.py", "AdjustedRandScore", "Adjusted Rand score between two clusterings.", [
        T, "from torchmetrics_forked_amd.clustering import AdjustedRandScore",
        "AdjustedRandScore()(torch.tensor([0, 0, 1, 1]), torch.tensor([0, 0, 1, 2]))"]),
    ("audio/_modules.py", "SignalNoiseRatio", "Signal-to-noise ratio.", [
        T, "from torchmetrics_forked_amd.audio import SignalNoiseRatio",
        "SignalNoiseRatio()(torch.tensor([2.5, 0.0, 2.0, 8.0]), torch.tensor([3.0, -0.5, 2.0, 7.0]))"]),
    ("audio/_modules.py", "ScaleInvariantSignalDistortionRatio", "Scale-invariant signal-to-distortion ratio.", [
        T, "from torchmetrics_forked_amd.audio import ScaleInvariantSignalDistortionRatio",
        "ScaleInvariantSignalDistortionRatio()(torch.tensor([2.5, 0.0, 2.0, 8.0]), torch.tensor([3.0, -0.5, 2.0, 7.0]))"]),
    ("image/_simple.py", "PeakSignalNoiseRatio", "Peak signal-to-noise ratio.", [
        T, "from torchmetrics_forked_amd.image import PeakSignalNoiseRatio",
        "PeakSignalNoiseRatio()(torch.tensor([[0.0, 1.0], [2.0, 3.0]]), torch.tensor([[3.0, 2.0], [1.0, 0.0]]))"]),
    ("nominal/_modules.py", "CramersV", "Cramer's V association between two categorical series.", [
        T, "from torchmetrics_forked_amd.nominal import CramersV",
        "CramersV(num_classes=3)(torch.tensor([0, 1, 2, 2, 1, 0, 1, 2]), torch.tensor([0, 1, 2, 1, 1, 0, 0, 2]))"]),
]

BP = "preds = torch.tensor([0.1, 0.8, 0.6, 0.3, 0.9, 0.2])"
BT = "target = torch.tensor([0, 1, 0, 0, 1, 1])"
MP = "preds = torch.tensor([2, 1, 0, 1, 2, 0])"
MT = "target = torch.tensor([2, 1, 0, 0, 1, 0])"
LP = "preds = torch.tensor([[0.2, 0.9, 0.1], [0.7, 0.4, 0.3], [0.6, 0.8, 0.9]])"
LT = "target = torch.tensor([[0, 1, 0], [1, 0, 1], [1, 1, 0]])"
RP = "preds = torch.tensor([2.5, 0.0, 2.0, 8.0, 4.2])"
RT = "target = torch.tensor([3.0, 0.5, 2.0, 7.0, 4.0])"


def _bin(cls, call="metric(preds, target)", kw=""):
    return ("classification", cls, f"{cls} (binary task).", [T, f"from torchmetrics_forked_amd.classification import {cls}", BP, BT,
                                                               f"metric = {cls}({kw})", call])


def _mc(cls, kw="num_classes=3", call="metric(preds, target)"):
    return ("classification", cls, f"{cls} (multiclass task).", [T, f"from torchmetrics_forked_amd.classification import {cls}", MP, MT,
                                                                   f"metric = {cls}({kw})", call])


def _ml(cls, kw="num_labels=3", call="metric(preds, target)"):
    return ("classification", cls, f"{cls} (multilabel task).", [T, f"from torchmetrics_forked_amd.classification import {cls}", LP, LT,
                                                                   f"metric = {cls}({kw})", call])


def _reg(cls, call="metric(preds, target)", kw="", pre=()):
    return ("regression", cls, f"{cls}.", [T, f"from torchmetrics_forked_amd.regression import {cls}", *pre, RP, RT, f"metric = {cls}({kw})", call])


def _clu(cls, kw=""):
    return ("clustering", cls, f"{cls}.", [T, f"from torchmetrics_forked_amd.clustering import {cls}",
                                           "preds = torch.tensor([2, 1, 0, 1, 0, 2])", "target = torch.tensor([0, 2, 1, 1, 0, 2])",
                                           f"{cls}({kw})(preds, target)"])


def _ret(cls, kw=""):
    return ("retrieval", cls, f"{cls} over queries.", [T, f"from torchmetrics_forked_amd.retrieval import {cls}",
                                                       "indexes = torch.tensor([0, 0, 0, 1, 1, 1, 1])",
                                                       "preds = torch.tensor([0.2, 0.3, 0.5, 0.1, 0.3, 0.5, 0.2])",
                                                       "target = torch.tensor([False, False, True, False, True, False, True])",
                                                       f"{cls}({kw})(preds, target, indexes=indexes)"])


SPECS += [
    _bin("BinaryF1Score"), _bin("BinaryPrecision"), _bin("BinaryRecall"), _bin("BinarySpecificity"), _bin("BinaryConfusionMatrix"),
    _bin("BinaryAveragePrecision"), _bin("BinaryCalibrationError", kw="n_bins=2"), _bin("BinaryHingeLoss"), _bin("BinaryCohenKappa"),
    _bin("BinaryMatthewsCorrCoef"), _bin("BinaryJaccardIndex"), _bin("BinaryStatScores"), _bin("BinaryHammingDistance"),
    _bin("BinaryFBetaScore", kw="beta=2.0"), _bin("BinaryPrecisionAtFixedRecall", kw="min_recall=0.5"),
    _bin("BinaryRecallAtFixedPrecision", kw="min_precision=0.5"), _bin("BinarySpecificityAtSensitivity", kw="min_sensitivity=0.5"),
    _mc("MulticlassHammingDistance"), _mc("MulticlassFBetaScore", kw="num_classes=3, beta=0.5"), _mc("MulticlassExactMatch", call="metric(preds.reshape(2, 3), target.reshape(2, 3))"),
    _ml("MultilabelF1Score"), _ml("MultilabelPrecision"), _ml("MultilabelRecall"), _ml("MultilabelAUROC", kw="num_labels=3, average=None"),
    _ml("MultilabelConfusionMatrix"), _ml("MultilabelCoverageError"), _ml("MultilabelRankingAveragePrecision"), _ml("MultilabelHammingDistance"),
    _ml("MultilabelAveragePrecision", kw="num_labels=3, average=None"), _ml("MultilabelExactMatch"), _ml("MultilabelStatScores", kw="num_labels=3, average=None"),
    _reg("MeanSquaredLogError"), _reg("MeanAbsolutePercentageError"), _reg("SymmetricMeanAbsolutePercentageError"),
    _reg("WeightedMeanAbsolutePercentageError"), _reg("LogCoshError"), _reg("MinkowskiDistance", kw="p=3"),
    _reg("TweedieDevianceScore", kw="power=0.0"), _reg("ConcordanceCorrCoef"), _reg("RelativeSquaredError"), _reg("CosineSimilarity", kw="reduction='mean'", call="metric(preds.reshape(1, -1), target.reshape(1, -1))"),
    ("regression", "KLDivergence", "KL divergence between distributions.", [T, "from torchmetrics_forked_amd.regression import KLDivergence",
        "p = torch.tensor([[0.36, 0.48, 0.16]])", "q = torch.tensor([[1 / 3, 1 / 3, 1 / 3]])", "KLDivergence()(p, q)"]),
    _clu("RandScore"), _clu("NormalizedMutualInfoScore"), _clu("AdjustedMutualInfoScore"), _clu("FowlkesMallowsIndex"),
    _clu("HomogeneityScore"), _clu("CompletenessScore"), _clu("VMeasureScore"),
    ("clustering", "CalinskiHarabaszScore", "Calinski-Harabasz score of a clustering.", [T, "from torchmetrics_forked_amd.clustering import CalinskiHarabaszScore",
        "data = torch.tensor([[0.0, 0.1], [0.2, 0.0], [5.0, 5.1], [5.2, 4.9], [9.9, 0.1], [10.1, 0.0]])", "labels = torch.tensor([0, 0, 1, 1, 2, 2])",
        "CalinskiHarabaszScore()(data, labels)"]),
    ("clustering", "DaviesBouldinScore", "Davies-Bouldin score of a clustering.", [T, "from torchmetrics_forked_amd.clustering import DaviesBouldinScore",
        "data = torch.tensor([[0.0, 0.1], [0.2, 0.0], [5.0, 5.1], [5.2, 4.9], [9.9, 0.1], [10.1, 0.0]])", "labels = torch.tensor([0, 0, 1, 1, 2, 2])",
        "DaviesBouldinScore()(data, labels)"]),
    _ret("RetrievalPrecision", kw="top_k=2"), _ret("RetrievalRecall", kw="top_k=2"), _ret("RetrievalFallOut", kw="top_k=2"),
    _ret("RetrievalHitRate", kw="top_k=2"), _ret("RetrievalRPrecision"),
    ("nominal", "TschuprowsT", "Tschuprow's T association.", [T, "from torchmetrics_forked_amd.nominal import TschuprowsT",
        "TschuprowsT(num_classes=3)(torch.tensor([0, 1, 2, 2, 1, 0, 1, 2]), torch.tensor([0, 1, 2, 1, 1, 0, 0, 2]))"]),
    ("nominal", "PearsonsContingencyCoefficient", "Pearson's contingency coefficient.", [T, "from torchmetrics_forked_amd.nominal import PearsonsContingencyCoefficient",
        "PearsonsContingencyCoefficient(num_classes=3)(torch.tensor([0, 1, 2, 2, 1, 0, 1, 2]), torch.tensor([0, 1, 2, 1, 1, 0, 0, 2]))"]),
    ("nominal", "TheilsU", "Theil's U (uncertainty coefficient).", [T, "from torchmetrics_forked_amd.nominal import TheilsU",
        "TheilsU(num_classes=3)(torch.tensor([0, 1, 2, 2, 1, 0, 1, 2]), torch.tensor([0, 1, 2, 1, 1, 0, 0, 2]))"]),
    ("text", "MatchErrorRate", "Match error rate.", ["from torchmetrics_forked_amd.text import MatchErrorRate",
        "MatchErrorRate()(['this is the prediction', 'there is an other sample'], ['this is the reference', 'there is another one'])"]),
    ("text", "WordInfoLost", "Word information lost.", ["from torchmetrics_forked_amd.text import WordInfoLost",
        "WordInfoLost()(['this is the prediction', 'there is an other sample'], ['this is the reference', 'there is another one'])"]),
    ("text", "CHRFScore", "chrF score of a corpus.", ["from torchmetrics_forked_amd.text import CHRFScore",
        "CHRFScore()(['the cat is on the mat'], [['there is a cat on the mat', 'a cat is on the mat']])"]),
    ("text", "TranslationEditRate", "Translation edit rate.", ["from torchmetrics_forked_amd.text import TranslationEditRate",
        "TranslationEditRate()(['the cat is on the mat'], [['there is a cat on the mat', 'a cat is on the mat']])"]),
    ("text", "SacreBLEUScore", "SacreBLEU score of a corpus.", ["from torchmetrics_forked_amd.text import SacreBLEUScore",
        "SacreBLEUScore()(['the squirrel is eating the nut'], [['a squirrel is eating a nut', 'the squirrel is eating a tasty nut']])"]),
    ("image", "StructuralSimilarityIndexMeasure", "Structural similarity index.", [T, "from torchmetrics_forked_amd.image import StructuralSimilarityIndexMeasure",
        "preds = torch.linspace(0, 1, 2 * 3 * 16 * 16).reshape(2, 3, 16, 16)", "target = preds.flip(-1) * 0.75",
        "StructuralSimilarityIndexMeasure(data_range=1.0)(preds, target)"]),
    ("image", "UniversalImageQualityIndex", "Universal image quality index.", [T, "from torchmetrics_forked_amd.image import UniversalImageQualityIndex",
        "preds = torch.linspace(0, 1, 2 * 3 * 16 * 16).reshape(2, 3, 16, 16)", "target = preds.flip(-1) * 0.75",
        "UniversalImageQualityIndex()(preds, target)"]),
    ("image", "TotalVariation", "Total variation of images.", [T, "from torchmetrics_forked_amd.image import TotalVariation",
        "img = torch.linspace(0, 1, 2 * 3 * 8 * 8).reshape(2, 3, 8, 8)", "TotalVariation()(img)"]),
    ("detection", "IntersectionOverUnion", "Box IoU for object detection.", [T, "from torchmetrics_forked_amd.detection import IntersectionOverUnion",
        "preds = [{'boxes': torch.tensor([[296.55, 93.96, 314.97, 152.79], [298.55, 98.96, 314.97, 151.79]]), 'labels': torch.tensor([4, 5])}]",
        "target = [{'boxes': torch.tensor([[300.00, 100.00, 315.00, 150.00]]), 'labels': torch.tensor([5])}]",
        "IntersectionOverUnion()(preds, target)"]),
    ("audio", "ScaleInvariantSignalNoiseRatio", "Scale-invariant signal-to-noise ratio.", [T, "from torchmetrics_forked_amd.audio import ScaleInvariantSignalNoiseRatio",
        RP, RT, "ScaleInvariantSignalNoiseRatio()(preds, target)"]),
    ("wrappers", "MinMaxMetric", "Tracks the min and max of a base metric's value.", [T, "from torchmetrics_forked_amd.wrappers import MinMaxMetric",
        "from torchmetrics_forked_amd.classification import BinaryAccuracy", "metric = MinMaxMetric(BinaryAccuracy())",
        "metric.update(torch.tensor([0.9, 0.2]), torch.tensor([1, 0]))", "metric.compute()",
        "metric.update(torch.tensor([0.9, 0.8]), torch.tensor([0, 0]))", "metric.compute()"]),
    ("wrappers", "ClasswiseWrapper", "Splits a per-class metric output into a dict.", [T, "from torchmetrics_forked_amd.wrappers import ClasswiseWrapper",
        "from torchmetrics_forked_amd.classification import MulticlassAccuracy",
        "metric = ClasswiseWrapper(MulticlassAccuracy(num_classes=3, average=None), labels=['cat', 'dog', 'fish'])",
        "metric(torch.tensor([2, 1, 0, 1]), torch.tensor([2, 1, 0, 0]))"]),
]


def _run(lines: List[str]) -> List[str]:
    """Execute the example lines; returns the doctest text (``>>>`` lines + expected outputs)."""
    ns: dict = {}
    out: List[str] = []
    for line in lines:
        out.append(f">>> {line}")
        try:
            code = compile(line, "<example>", "eval")
            is_expr = True
        except SyntaxError:
            code = compile(line, "<example>", "exec")
            is_expr = False
        buf = io.StringIO()
        with redirect_stdout(buf):
            res = eval(code, ns) if is_expr else exec(code, ns)  # noqa: S307 - our own example lines
        printed = buf.getvalue().rstrip("\n")
        if printed:
            out.extend(r if r.strip() else "<BLANKLINE>" for r in printed.splitlines())
        if is_expr and res is not None:
            out.extend(r if r.strip() else "<BLANKLINE>" for r in repr(res).splitlines())
    return out


def _class_block(src: str, name: str) -> Tuple[int, int, int]:
    """(class line index, docstring start index or -1, docstring end index) in ``src.splitlines()``."""
    tree = ast.parse(src)
    for node in ast.walk(tree):
        if isinstance(node, ast.ClassDef) and node.name == name:
            body0 = node.body[0]
            if isinstance(body0, ast.Expr) and isinstance(getattr(body0, "value", None), ast.Constant) and isinstance(body0.value.value, str):
                return node.lineno - 1, body0.lineno - 1, body0.end_lineno - 1
            return node.lineno - 1, -1, -1
    raise KeyError(name)


def patch(path: str, name: str, summary: str, lines: List[str], check: bool) -> bool:
    src = open(path).read()
    cls_i, d0, d1 = _class_block(src, name)
    rows = src.splitlines()
    if d0 >= 0 and any("Example:" in r for r in rows[d0 : d1 + 1]):
        return False
    if check:
        print(f"missing example: {name} ({os.path.relpath(path, ROOT)})")
        return True
    ind = " " * (len(rows[cls_i]) - len(rows[cls_i].lstrip()) + 4)
    example = [f"{ind}Example:"] + [f"{ind}    {r}" if r else "" for r in _run(lines)]
    if d0 < 0:
        new = [f'{ind}"""{summary}', ""] + example + [f'{ind}"""']
        rows[cls_i + 1 : cls_i + 1] = new
    elif d0 == d1:  # one-line docstring
        text = rows[d0].strip()
        q = text[:3]
        body = text[3:-3]
        rows[d0 : d0 + 1] = [f"{ind}{q}{body}", ""] + example + [f"{ind}{q}"]
    else:
        closing = rows[d1]
        if closing.strip() in ('"""', "'''"):
            rows[d1:d1] = [""] + example
        else:  # text and closing quotes on the last line
            q = closing.rstrip()[-3:]
            rows[d1] = closing.rstrip()[:-3]
            rows[d1 + 1 : d1 + 1] = [""] + example + [f"{ind}{q}"]
    open(path, "w").write("\n".join(rows) + ("\n" if src.endswith("\n") else ""))
    return True


def main() -> None:
    check = "--check" in sys.argv
    n = 0
    for rel, name, summary, lines in SPECS:
        import importlib
        import inspect

        mod = importlib.import_module("torchmetrics_forked_amd." + rel.split("/")[0].replace(".py", ""))
        path = inspect.getsourcefile(getattr(mod, name))  # the defining module (spec paths are only the domain)
        n += patch(path, name, summary, lines, check)
    print(f"{'missing' if check else 'patched'}: {n} of {len(SPECS)}")


if __name__ == "__main__":
    main()
