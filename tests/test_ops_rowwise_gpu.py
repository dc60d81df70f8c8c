"""gfx950 row kernels (csrc/rowwise.hip, csrc/clustering.hip) vs the eager CPU path of the same functions.

* top-k / samplewise multiclass stat scores: integer counts, exact (tie-free scores);
* multiclass hinge (crammer-singer / one-vs-all, squared, logits and probabilities): fp32 within float rounding,
  16-bit inputs within one rounding of the input dtype per row;
* multilabel coverage / LRAP / ranking loss: exact on integer-valued (tie-heavy) scores;
* expected mutual information (adjusted mutual info) in fp64.
"""
import pytest
import torch

import torchmetrics_forked_amd as tm
import torchmetrics_forked_amd.functional as F
from torchmetrics_forked_amd import ops

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_native(device):
    ops.require()


def _scores(shape, seed, dtype=torch.float32):
    g = torch.Generator().manual_seed(seed)
    # a random permutation per row: no ties in any dtype that holds the integers exactly
    n, c = shape[0], shape[1]
    rest = shape[2:]
    x = torch.rand(n, c, *rest, generator=g).argsort(dim=1).to(torch.float32) / c
    return x.to(dtype)


@pytest.mark.parametrize("C", [5, 64, 100, 1000, 2000])
@pytest.mark.parametrize("top_k", [1, 2, 5])
@pytest.mark.parametrize("average", ["micro", "macro", None])
@pytest.mark.parametrize("mdim", ["global", "samplewise"])
def test_topk_stat_scores_vs_cpu(C, top_k, average, mdim):
    if top_k > C:
        pytest.skip("top_k > C")
    n, x = 257, (3 if mdim == "samplewise" else 1)
    p = _scores((n, C, x), C + top_k).squeeze(-1) if x == 1 else _scores((n, C, x), C + top_k)
    g = torch.Generator().manual_seed(7)
    t = torch.randint(0, C, (n, x) if x > 1 else (n,), generator=g)
    kw = dict(num_classes=C, top_k=top_k, average=average, multidim_average=mdim)
    cpu = F.multiclass_stat_scores(p, t, **kw)
    gpu = F.multiclass_stat_scores(p.cuda(), t.cuda(), **kw).cpu()
    _same(gpu, cpu)


def _same(gpu, cpu):
    if cpu.is_floating_point():  # macro / weighted means: float reduction order may differ
        torch.testing.assert_close(gpu, cpu, rtol=1e-6, atol=1e-6)
    else:
        assert torch.equal(gpu, cpu)


@pytest.mark.parametrize("ignore_index", [0, -1, 7])
@pytest.mark.parametrize("mdim", ["global", "samplewise"])
def test_topk_stat_scores_ignore_index(ignore_index, mdim):
    C, n = 10, 300
    p = _scores((n, C, 4), 3)
    g = torch.Generator().manual_seed(8)
    t = torch.randint(0, C, (n, 4), generator=g)
    t[::5, 1] = ignore_index
    for k in (1, 3):
        kw = dict(num_classes=C, top_k=k, average=None, multidim_average=mdim, ignore_index=ignore_index)
        cpu = F.multiclass_stat_scores(p, t, **kw)
        gpu = F.multiclass_stat_scores(p.cuda(), t.cuda(), **kw).cpu()
        _same(gpu, cpu)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
def test_topk_accuracy_module_matches_cpu(dtype):
    C, n = 1000, 4096
    p = _scores((n, C), 11, dtype=torch.float32).to(dtype)
    t = torch.randint(0, C, (n,), generator=torch.Generator().manual_seed(12))
    for cls in (tm.classification.MulticlassAccuracy, tm.classification.MulticlassF1Score, tm.classification.MulticlassRecall):
        mc, mg = cls(num_classes=C, top_k=5), cls(num_classes=C, top_k=5).cuda()
        for s in range(0, n, 1024):
            mc.update(p[s : s + 1024], t[s : s + 1024])
            mg.update(p[s : s + 1024].cuda(), t[s : s + 1024].cuda())
        torch.testing.assert_close(mg.compute().cpu(), mc.compute(), rtol=1e-6, atol=1e-7)


def test_topk_nan_rows_follow_topk_order():
    """NaN is ordered before every number (torch.topk): a NaN entry is always picked first."""
    C, n = 20, 64
    p = _scores((n, C), 5)
    p[::3, 4] = float("nan")
    t = torch.full((n,), 4, dtype=torch.long)
    out = F.multiclass_stat_scores(p.cuda(), t.cuda(), num_classes=C, top_k=2, average=None).cpu()
    assert int(out[4, 0]) >= (n + 2) // 3  # every NaN row is a tp for class 4


@pytest.mark.parametrize("mode", ["crammer-singer", "one-vs-all"])
@pytest.mark.parametrize("squared", [False, True])
@pytest.mark.parametrize("probs", [False, True])
@pytest.mark.parametrize("C", [3, 100, 1000])
def test_mc_hinge_vs_cpu_fp32(mode, squared, probs, C):
    g = torch.Generator().manual_seed(C)
    x = torch.randn(2000, C, generator=g)
    if probs:
        x = x.softmax(1)
    t = torch.randint(0, C, (2000,), generator=g)
    cpu = F.multiclass_hinge_loss(x, t, C, squared=squared, multiclass_mode=mode)
    gpu = F.multiclass_hinge_loss(x.cuda(), t.cuda(), C, squared=squared, multiclass_mode=mode).cpu()
    torch.testing.assert_close(gpu, cpu, rtol=2e-5, atol=1e-6)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("mode", ["crammer-singer", "one-vs-all"])
def test_mc_hinge_16bit(dtype, mode):
    C = 50
    g = torch.Generator().manual_seed(3)
    x = torch.randn(1000, C, generator=g).to(dtype)
    t = torch.randint(0, C, (1000,), generator=g)
    m = tm.classification.MulticlassHingeLoss(num_classes=C, multiclass_mode=mode).cuda()
    m.update(x.cuda(), t.cuda())
    ref = F.multiclass_hinge_loss(x.float().cuda(), t.cuda(), C, multiclass_mode=mode).cpu()
    # per-element rounding to the input dtype: within a few units of its epsilon of the fp32 value
    tol = 4 * torch.finfo(dtype).eps
    torch.testing.assert_close(m.compute().cpu().float(), ref, rtol=tol, atol=tol)


@pytest.mark.parametrize("L", [5, 64, 300, 1500])
@pytest.mark.parametrize("metric", ["coverage", "lrap", "loss"])
@pytest.mark.parametrize("ties", [False, True])
def test_multilabel_ranking_vs_cpu(L, metric, ties):
    g = torch.Generator().manual_seed(L)
    n = 777
    x = torch.randint(0, 6, (n, L), generator=g).float() if ties else torch.randn(n, L, generator=g)
    t = torch.randint(0, 2, (n, L), generator=g)
    t[0] = 0  # degenerate rows: nothing relevant / everything relevant
    t[1] = 1
    fn = {"coverage": F.multilabel_coverage_error, "lrap": F.multilabel_ranking_average_precision,
          "loss": F.multilabel_ranking_loss}[metric]
    cpu = fn(x, t, num_labels=L)
    gpu = fn(x.cuda(), t.cuda(), num_labels=L).cpu()
    torch.testing.assert_close(gpu, cpu, rtol=1e-5, atol=1e-6)


def test_multilabel_ranking_loss_all_degenerate():
    x = torch.randn(10, 4).cuda()
    t = torch.zeros(10, 4, dtype=torch.long).cuda()
    assert float(F.multilabel_ranking_loss(x, t, num_labels=4)) == 0.0


@pytest.mark.parametrize("n,kp,kt", [(1000, 5, 7), (20000, 40, 30), (300, 300, 2)])
def test_adjusted_mutual_info_gpu_vs_cpu(n, kp, kt):
    g = torch.Generator().manual_seed(n)
    p = torch.randint(0, kp, (n,), generator=g)
    t = torch.randint(0, kt, (n,), generator=g)
    cpu = F.clustering.adjusted_mutual_info_score(p, t)
    gpu = F.clustering.adjusted_mutual_info_score(p.cuda(), t.cuda()).cpu()
    torch.testing.assert_close(gpu, cpu, rtol=1e-5, atol=1e-6)


def test_expected_mutual_info_kernel_vs_fp64_oracle():
    from torchmetrics_forked_amd.functional.clustering.adjusted_mutual_info_score import expected_mutual_info_score
    from torchmetrics_forked_amd.ops.clustering import expected_mutual_info

    g = torch.Generator().manual_seed(0)
    cont = torch.randint(0, 50, (9, 13), generator=g)
    n = int(cont.sum())
    ref = expected_mutual_info_score(cont, n).double()  # CPU: masked fp64 tensor expression
    got = expected_mutual_info(cont.sum(1).double().cuda(), cont.sum(0).double().cuda(), n).cpu()
    assert abs(float(got) - float(ref)) <= 1e-6 * max(1.0, abs(float(ref)))


@pytest.mark.parametrize("C", [3, 17, 200])
@pytest.mark.parametrize("kind", ["roc", "pr"])
def test_macro_curve_interp_gpu_vs_cpu(C, kind):
    """Macro-averaged ROC / PR curves: one csrc/interp.hip launch over all classes vs the per-class interp loop."""
    g = torch.Generator().manual_seed(C)
    x = torch.randn(3000, C, generator=g).softmax(1)
    x = (x * 50).round() / 50  # ties: repeated curve points and zero-width segments
    t = torch.randint(0, C, (3000,), generator=g)
    fn = F.multiclass_roc if kind == "roc" else F.multiclass_precision_recall_curve
    for thresholds in (None, 50):
        cpu = fn(x, t, num_classes=C, average="macro", thresholds=thresholds)
        gpu = fn(x.cuda(), t.cuda(), num_classes=C, average="macro", thresholds=thresholds)
        for a, b in zip(gpu, cpu):
            torch.testing.assert_close(a.cpu(), b, rtol=1e-6, atol=1e-6)
