"""MetricTester-depth matrix over the domains (reference strategy: every metric runs through ddp x
dist_sync_on_step x pickle / clone / state attributes, reduced precision, differentiability and TorchScript;
``tests/unittests/helpers/testers.py:74-227,285-317,454-520``).

Each case is (module class, functional, oracle, data, kwargs).  The oracle is the reference functional where the
reference runs in this image, otherwise this framework's own functional (module-vs-functional consistency; noted
as "self" below)."""
import pytest
import torch

import torchmetrics_forked_amd as tm
import torchmetrics_forked_amd.functional as F
from tests.helpers.testers import (
    BATCH_SIZE,
    NUM_BATCHES,
    NUM_CLASSES,
    RefFn,
    run_class_metric_test,
    run_differentiability_test,
    run_precision_test,
    run_scriptable_test,
)

_g = torch.Generator().manual_seed(1234)
BIN = (torch.rand(NUM_BATCHES, BATCH_SIZE, generator=_g), torch.randint(0, 2, (NUM_BATCHES, BATCH_SIZE), generator=_g))
MC = (torch.randn(NUM_BATCHES, BATCH_SIZE, NUM_CLASSES, generator=_g), torch.randint(0, NUM_CLASSES, (NUM_BATCHES, BATCH_SIZE), generator=_g))
ML = (torch.rand(NUM_BATCHES, BATCH_SIZE, NUM_CLASSES, generator=_g), torch.randint(0, 2, (NUM_BATCHES, BATCH_SIZE, NUM_CLASSES), generator=_g))
REG = (torch.randn(NUM_BATCHES, BATCH_SIZE, generator=_g), torch.randn(NUM_BATCHES, BATCH_SIZE, generator=_g))
POS = (torch.rand(NUM_BATCHES, BATCH_SIZE, generator=_g) + 0.1, torch.rand(NUM_BATCHES, BATCH_SIZE, generator=_g) + 0.1)
IMG = (torch.rand(NUM_BATCHES, 2, 3, 24, 24, generator=_g), torch.rand(NUM_BATCHES, 2, 3, 24, 24, generator=_g))

K = NUM_CLASSES
CASES = {
    "binary_accuracy": (tm.classification.BinaryAccuracy, F.classification.binary_accuracy, RefFn("binary_accuracy"), BIN, {}),
    "multiclass_f1": (tm.classification.MulticlassF1Score, F.classification.multiclass_f1_score,
                      RefFn("multiclass_f1_score", num_classes=K), MC, {"num_classes": K}),
    "multilabel_precision": (tm.classification.MultilabelPrecision, F.classification.multilabel_precision,
                             RefFn("multilabel_precision", num_labels=K), ML, {"num_labels": K}),
    "multiclass_auroc": (tm.classification.MulticlassAUROC, F.classification.multiclass_auroc,
                         RefFn("multiclass_auroc", num_classes=K), MC, {"num_classes": K}),
    "binary_average_precision": (tm.classification.BinaryAveragePrecision, F.classification.binary_average_precision,
                                 RefFn("binary_average_precision"), BIN, {}),
    "multiclass_confusion_matrix": (tm.classification.MulticlassConfusionMatrix, F.classification.multiclass_confusion_matrix,
                                    RefFn("multiclass_confusion_matrix", num_classes=K), MC, {"num_classes": K}),
    "multiclass_calibration_error": (tm.classification.MulticlassCalibrationError, F.classification.multiclass_calibration_error,
                                     RefFn("multiclass_calibration_error", num_classes=K), MC, {"num_classes": K}),
    "binary_hinge": (tm.classification.BinaryHingeLoss, F.classification.binary_hinge_loss, RefFn("binary_hinge_loss"), BIN, {}),
    "mse": (tm.regression.MeanSquaredError, F.regression.mean_squared_error, RefFn("mean_squared_error", "regression"), REG, {}),
    "mae": (tm.regression.MeanAbsoluteError, F.regression.mean_absolute_error, RefFn("mean_absolute_error", "regression"), REG, {}),
    "pearson": (tm.regression.PearsonCorrCoef, F.regression.pearson_corrcoef, RefFn("pearson_corrcoef", "regression"), REG, {}),
    "r2": (tm.regression.R2Score, F.regression.r2_score, RefFn("r2_score", "regression"), REG, {}),
    "spearman": (tm.regression.SpearmanCorrCoef, F.regression.spearman_corrcoef, RefFn("spearman_corrcoef", "regression"), REG, {}),
    "explained_variance": (tm.regression.ExplainedVariance, F.regression.explained_variance,
                           RefFn("explained_variance", "regression"), REG, {}),
    "mape": (tm.regression.MeanAbsolutePercentageError, F.regression.mean_absolute_percentage_error,
             RefFn("mean_absolute_percentage_error", "regression"), POS, {}),
    "log_cosh": (tm.regression.LogCoshError, F.regression.log_cosh_error, RefFn("log_cosh_error", "regression"), REG, {}),
    "psnr": (tm.image.PeakSignalNoiseRatio, F.image.peak_signal_noise_ratio,
             RefFn("peak_signal_noise_ratio", "image", data_range=1.0), IMG, {"data_range": 1.0}),
    "ssim": (tm.image.StructuralSimilarityIndexMeasure, F.image.structural_similarity_index_measure,
             RefFn("structural_similarity_index_measure", "image", data_range=1.0), IMG, {"data_range": 1.0}),
}


@pytest.mark.parametrize("dist_sync_on_step", [False, True])
@pytest.mark.parametrize("ddp", [False, True])
@pytest.mark.parametrize("name", sorted(CASES))
def test_ddp_sync_on_step_matrix(reference, name, ddp, dist_sync_on_step):
    if not ddp and dist_sync_on_step:
        pytest.skip("dist_sync_on_step is a no-op without a process group")
    cls, _, oracle, (p, t), kw = CASES[name]
    atol = 1e-4 if name in ("ssim", "multiclass_calibration_error", "explained_variance", "r2", "pearson") else 1e-6
    run_class_metric_test(ddp, p, t, cls, oracle, kw, dist_sync_on_step=dist_sync_on_step, atol=atol)


PRECISION = ["binary_accuracy", "multiclass_f1", "multiclass_auroc", "mse", "mae", "pearson", "psnr"]


@pytest.mark.parametrize("dtype", [torch.half, torch.bfloat16])
@pytest.mark.parametrize("name", PRECISION)
def test_reduced_precision(name, dtype):
    cls, fn, _, (p, t), kw = CASES[name]
    run_precision_test(p, t, cls, fn, kw, dtype=dtype, atol=6e-2)


@pytest.mark.parametrize("name", sorted(CASES))
def test_differentiability(name):
    cls, fn, _, (p, t), kw = CASES[name]
    run_differentiability_test(p, t, cls, fn, kw)


@pytest.mark.parametrize("name", ["binary_accuracy", "multiclass_f1", "mse", "mae", "pearson", "r2", "psnr"])
def test_scriptable(name):
    cls, _, _, (p, t), kw = CASES[name]
    run_scriptable_test(cls, p, t, kw)


class _SelfOracle:
    """This framework's functional on CPU (the GPU box has no reference tree): module-on-GPU vs functional-on-CPU."""

    def __init__(self, fn, kw):
        self.fn, self.kw = fn, kw

    def __call__(self, p, t):
        return self.fn(p, t, **self.kw)


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(CASES))
def test_gpu_module_matrix(name):
    """Every case with GPU-resident states (native update paths) against the CPU functional, batch and final values,
    plus reduced-precision inputs on the GPU."""
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    cls, fn, _, (p, t), kw = CASES[name]
    atol = 1e-4 if name in ("ssim", "multiclass_calibration_error", "explained_variance", "r2", "pearson", "spearman") else 1e-5
    run_class_metric_test(False, p, t, cls, _SelfOracle(fn, kw), kw, atol=atol, device="cuda")
    if name in PRECISION:
        run_precision_test(p, t, cls, fn, kw, dtype=torch.bfloat16, device="cuda", atol=6e-2)
