"""Module-level classification tests: batch forward values, accumulation across batches and 2-process gloo
sync (coalesced all-reduce for sum states, packed gather for cat states), against the reference functional."""
import importlib

import pytest
import torch

import torchmetrics_forked_amd.classification as C
from tests.helpers.testers import BATCH_SIZE, NUM_BATCHES, NUM_CLASSES, RefFn, run_class_metric_test

_g = torch.Generator().manual_seed(42)
BIN = (torch.rand(NUM_BATCHES, BATCH_SIZE, generator=_g), torch.randint(0, 2, (NUM_BATCHES, BATCH_SIZE), generator=_g))
MC = (torch.randn(NUM_BATCHES, BATCH_SIZE, NUM_CLASSES, generator=_g), torch.randint(0, NUM_CLASSES, (NUM_BATCHES, BATCH_SIZE), generator=_g))
ML = (torch.rand(NUM_BATCHES, BATCH_SIZE, NUM_CLASSES, generator=_g), torch.randint(0, 2, (NUM_BATCHES, BATCH_SIZE, NUM_CLASSES), generator=_g))
MC16 = (MC[0].bfloat16(), MC[1])


def _ref(reference, name, **kw):
    return RefFn(name, "classification", **kw)


STAT = [("Accuracy", "accuracy"), ("Precision", "precision"), ("Recall", "recall"), ("Specificity", "specificity"),
        ("HammingDistance", "hamming_distance"), ("F1Score", "f1_score"), ("StatScores", "stat_scores")]


@pytest.mark.parametrize("ddp", [False, True])
@pytest.mark.parametrize("cls_name,fn", STAT)
def test_stat_family_modules(reference, ddp, cls_name, fn):
    run_class_metric_test(ddp, *BIN, getattr(C, f"Binary{cls_name}"), _ref(reference, f"binary_{fn}"))
    for avg in ("micro", "macro", "none"):
        run_class_metric_test(ddp, *MC, getattr(C, f"Multiclass{cls_name}"), _ref(reference, f"multiclass_{fn}", num_classes=NUM_CLASSES, average=avg),
                              {"num_classes": NUM_CLASSES, "average": avg})
        run_class_metric_test(ddp, *ML, getattr(C, f"Multilabel{cls_name}"), _ref(reference, f"multilabel_{fn}", num_labels=NUM_CLASSES, average=avg),
                              {"num_labels": NUM_CLASSES, "average": avg})


@pytest.mark.parametrize("ddp", [False, True])
def test_samplewise_cat_states(reference, ddp):
    p, t = torch.rand(NUM_BATCHES, BATCH_SIZE, 3, generator=_g), torch.randint(0, 2, (NUM_BATCHES, BATCH_SIZE, 3), generator=_g)
    run_class_metric_test(ddp, p, t, C.BinaryAccuracy, _ref(reference, "binary_accuracy", multidim_average="samplewise"),
                          {"multidim_average": "samplewise"})


CURVES = [("AUROC", "auroc"), ("AveragePrecision", "average_precision"), ("ROC", "roc"), ("PrecisionRecallCurve", "precision_recall_curve")]


@pytest.mark.parametrize("ddp", [False, True])
@pytest.mark.parametrize("thresholds", [None, 11])
@pytest.mark.parametrize("cls_name,fn", CURVES)
def test_curve_modules(reference, ddp, thresholds, cls_name, fn):
    atol = 1e-5
    run_class_metric_test(ddp, *BIN, getattr(C, f"Binary{cls_name}"), _ref(reference, f"binary_{fn}", thresholds=thresholds),
                          {"thresholds": thresholds}, atol=atol)
    for data in (MC, MC16):
        run_class_metric_test(ddp, *data, getattr(C, f"Multiclass{cls_name}"),
                              _ref(reference, f"multiclass_{fn}", num_classes=NUM_CLASSES, thresholds=thresholds),
                              {"num_classes": NUM_CLASSES, "thresholds": thresholds}, atol=atol)
    run_class_metric_test(ddp, *ML, getattr(C, f"Multilabel{cls_name}"), _ref(reference, f"multilabel_{fn}", num_labels=NUM_CLASSES, thresholds=thresholds),
                          {"num_labels": NUM_CLASSES, "thresholds": thresholds}, atol=atol)


@pytest.mark.parametrize("ddp", [False, True])
def test_confusion_matrix_modules(reference, ddp):
    run_class_metric_test(ddp, *BIN, C.BinaryConfusionMatrix, _ref(reference, "binary_confusion_matrix"))
    run_class_metric_test(ddp, *MC, C.MulticlassConfusionMatrix, _ref(reference, "multiclass_confusion_matrix", num_classes=NUM_CLASSES),
                          {"num_classes": NUM_CLASSES})
    run_class_metric_test(ddp, *ML, C.MultilabelConfusionMatrix, _ref(reference, "multilabel_confusion_matrix", num_labels=NUM_CLASSES),
                          {"num_labels": NUM_CLASSES})


def test_task_wrappers():
    assert isinstance(C.Accuracy(task="binary"), C.BinaryAccuracy)
    assert isinstance(C.AUROC(task="multiclass", num_classes=3), C.MulticlassAUROC)
    assert isinstance(C.F1Score(task="multilabel", num_labels=3), C.MultilabelF1Score)
    assert isinstance(C.ConfusionMatrix(task="multiclass", num_classes=3), C.MulticlassConfusionMatrix)
    with pytest.raises(ValueError):
        C.Accuracy(task="multiclass")
    with pytest.raises(ValueError, match="Invalid Classification"):
        C.Accuracy(task="foo")
