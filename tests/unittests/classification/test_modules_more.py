"""Module + 2-process DDP tests for the second batch of classification metrics vs the reference functional."""
import pytest
import torch

import torchmetrics_forked_amd.classification as C
from tests.helpers.testers import BATCH_SIZE, NUM_BATCHES, NUM_CLASSES, RefFn, assert_allclose, run_class_metric_test

_g = torch.Generator().manual_seed(7)
BIN = (torch.rand(NUM_BATCHES, BATCH_SIZE, generator=_g), torch.randint(0, 2, (NUM_BATCHES, BATCH_SIZE), generator=_g))
MC = (torch.randn(NUM_BATCHES, BATCH_SIZE, NUM_CLASSES, generator=_g), torch.randint(0, NUM_CLASSES, (NUM_BATCHES, BATCH_SIZE), generator=_g))
ML = (torch.rand(NUM_BATCHES, BATCH_SIZE, NUM_CLASSES, generator=_g), torch.randint(0, 2, (NUM_BATCHES, BATCH_SIZE, NUM_CLASSES), generator=_g))
NC = NUM_CLASSES


def R(name, **kw):
    return RefFn(name, "classification", **kw)


@pytest.mark.parametrize("ddp", [False, True])
def test_confmat_derived(ddp):
    run_class_metric_test(ddp, *BIN, C.BinaryCohenKappa, R("binary_cohen_kappa"))
    run_class_metric_test(ddp, *MC, C.MulticlassCohenKappa, R("multiclass_cohen_kappa", num_classes=NC, weights="quadratic"),
                          {"num_classes": NC, "weights": "quadratic"})
    run_class_metric_test(ddp, *BIN, C.BinaryMatthewsCorrCoef, R("binary_matthews_corrcoef"))
    run_class_metric_test(ddp, *MC, C.MulticlassMatthewsCorrCoef, R("multiclass_matthews_corrcoef", num_classes=NC), {"num_classes": NC})
    run_class_metric_test(ddp, *ML, C.MultilabelMatthewsCorrCoef, R("multilabel_matthews_corrcoef", num_labels=NC), {"num_labels": NC})
    run_class_metric_test(ddp, *BIN, C.BinaryJaccardIndex, R("binary_jaccard_index"))
    for avg in ("macro", "micro", "none"):
        run_class_metric_test(ddp, *MC, C.MulticlassJaccardIndex, R("multiclass_jaccard_index", num_classes=NC, average=avg),
                              {"num_classes": NC, "average": avg})
        run_class_metric_test(ddp, *ML, C.MultilabelJaccardIndex, R("multilabel_jaccard_index", num_labels=NC, average=avg),
                              {"num_labels": NC, "average": avg})


@pytest.mark.parametrize("ddp", [False, True])
def test_exact_match_hinge_calibration(ddp):
    X = 3
    mc3 = (torch.randint(0, NC, (NUM_BATCHES, BATCH_SIZE, X), generator=_g), torch.randint(0, NC, (NUM_BATCHES, BATCH_SIZE, X), generator=_g))
    mc3 = (torch.where(torch.rand(mc3[0].shape, generator=_g) < 0.6, mc3[1], mc3[0]), mc3[1])
    run_class_metric_test(ddp, *mc3, C.MulticlassExactMatch, R("multiclass_exact_match", num_classes=NC), {"num_classes": NC})
    run_class_metric_test(ddp, *mc3, C.MulticlassExactMatch, R("multiclass_exact_match", num_classes=NC, multidim_average="samplewise"),
                          {"num_classes": NC, "multidim_average": "samplewise"})
    run_class_metric_test(ddp, *ML, C.MultilabelExactMatch, R("multilabel_exact_match", num_labels=NC), {"num_labels": NC})
    run_class_metric_test(ddp, *BIN, C.BinaryHingeLoss, R("binary_hinge_loss", squared=True), {"squared": True}, atol=1e-5)
    for mode in ("crammer-singer", "one-vs-all"):
        run_class_metric_test(ddp, *MC, C.MulticlassHingeLoss, R("multiclass_hinge_loss", num_classes=NC, multiclass_mode=mode),
                              {"num_classes": NC, "multiclass_mode": mode}, atol=1e-5)
    for norm in ("l1", "l2", "max"):
        run_class_metric_test(ddp, *BIN, C.BinaryCalibrationError, R("binary_calibration_error", norm=norm), {"norm": norm}, atol=1e-5)
        run_class_metric_test(ddp, *MC, C.MulticlassCalibrationError, R("multiclass_calibration_error", num_classes=NC, norm=norm),
                              {"num_classes": NC, "norm": norm}, atol=1e-5)


@pytest.mark.parametrize("ddp", [False, True])
@pytest.mark.parametrize("cls_name,fn", [("MultilabelCoverageError", "multilabel_coverage_error"),
                                          ("MultilabelRankingAveragePrecision", "multilabel_ranking_average_precision"),
                                          ("MultilabelRankingLoss", "multilabel_ranking_loss")])
def test_ranking_modules(ddp, cls_name, fn):
    run_class_metric_test(ddp, *ML, getattr(C, cls_name), R(fn, num_labels=NC), {"num_labels": NC}, atol=1e-5)


FIXED = [("RecallAtFixedPrecision", "recall_at_fixed_precision", "min_precision"),
         ("PrecisionAtFixedRecall", "precision_at_fixed_recall", "min_recall"),
         ("SpecificityAtSensitivity", "specificity_at_sensitivity", "min_sensitivity")]


@pytest.mark.parametrize("ddp", [False, True])
@pytest.mark.parametrize("thresholds", [None, 11])
@pytest.mark.parametrize("cls_name,fn,arg", FIXED)
def test_fixed_point_modules(ddp, thresholds, cls_name, fn, arg):
    kw = {arg: 0.5, "thresholds": thresholds}
    run_class_metric_test(ddp, *BIN, getattr(C, f"Binary{cls_name}"), R(f"binary_{fn}", **kw), kw, atol=1e-5)
    run_class_metric_test(ddp, *MC, getattr(C, f"Multiclass{cls_name}"), R(f"multiclass_{fn}", num_classes=NC, **kw),
                          {"num_classes": NC, **kw}, atol=1e-5)
    run_class_metric_test(ddp, *ML, getattr(C, f"Multilabel{cls_name}"), R(f"multilabel_{fn}", num_labels=NC, **kw),
                          {"num_labels": NC, **kw}, atol=1e-5)


def test_fixed_point_task_wrappers():
    m = C.RecallAtFixedPrecision("multiclass", 0.3, num_classes=3)
    assert isinstance(m, C.MulticlassRecallAtFixedPrecision) and m.min_precision == 0.3
    m = C.PrecisionAtFixedRecall("binary", min_recall=0.2, thresholds=5)
    assert isinstance(m, C.BinaryPrecisionAtFixedRecall) and m.thresholds.numel() == 5
    m = C.SpecificityAtSensitivity("multilabel", 0.4, None, None, 4)
    assert isinstance(m, C.MultilabelSpecificityAtSensitivity) and m.num_labels == 4
    with pytest.raises(TypeError):
        C.RecallAtFixedPrecision("binary")


def test_group_fairness_modules(reference):
    Rf = reference.functional.classification
    g = torch.Generator().manual_seed(3)
    ps = [torch.rand(40, generator=g) for _ in range(3)]
    ts = [torch.randint(0, 2, (40,), generator=g) for _ in range(3)]
    gs = [torch.arange(40) % 3 for _ in range(3)]  # every batch holds every group
    m = C.BinaryGroupStatRates(num_groups=3)
    f = C.BinaryFairness(num_groups=3)
    for p, t, gr in zip(ps, ts, gs):
        m.update(p, t, gr)
        f.update(p, t, gr)
    P, T, G = torch.cat(ps), torch.cat(ts), torch.cat(gs)
    assert_allclose(m.compute(), Rf.binary_groups_stat_rates(P, T, G, 3))
    res, ref = f.compute(), Rf.binary_fairness(P, T, G, "all")
    assert res.keys() == ref.keys()
    assert_allclose(res, ref)
    dp = C.BinaryFairness(num_groups=3, task="demographic_parity")
    dp.update(P, None, G)
    assert_allclose(dp.compute(), Rf.demographic_parity(P, G))


@pytest.mark.parametrize("ddp", [False, True])
def test_dice_module(ddp):
    run_class_metric_test(ddp, *MC, C.Dice, R("dice"), {})
    run_class_metric_test(ddp, *MC, C.Dice, R("dice", average="macro", num_classes=NC), {"average": "macro", "num_classes": NC})
    run_class_metric_test(ddp, *MC, C.Dice, R("dice", average="samples"), {"average": "samples"})


def test_metric_collection_fuses_confmat_subclasses(reference):
    """Kappa/MCC/Jaccard on the MulticlassConfusionMatrix state join the fused AUROC plan (bf16 scores)."""
    from torchmetrics_forked_amd import MetricCollection

    coll = MetricCollection({
        "auroc": C.MulticlassAUROC(NC),
        "kappa": C.MulticlassCohenKappa(NC),
        "mcc": C.MulticlassMatthewsCorrCoef(NC),
        "jac": C.MulticlassJaccardIndex(NC),
    })
    p, t = MC[0][0].bfloat16(), MC[1][0]
    coll.update(p, t)
    assert coll._fused_plans, "expected a fused plan"
    res = coll.compute()
    Rf = reference.functional.classification
    assert_allclose(res["kappa"], Rf.multiclass_cohen_kappa(p.float(), t, NC), 1e-6)
    assert_allclose(res["mcc"], Rf.multiclass_matthews_corrcoef(p.float(), t, NC), 1e-6)
    assert_allclose(res["jac"], Rf.multiclass_jaccard_index(p.float(), t, NC), 1e-6)
