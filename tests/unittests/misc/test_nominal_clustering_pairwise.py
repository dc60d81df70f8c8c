"""Nominal, clustering and pairwise parity vs the reference oracle (functional + modules + 2-process sync)."""
import pytest
import torch

import torchmetrics_forked_amd.clustering as CL
import torchmetrics_forked_amd.functional.clustering as FC
import torchmetrics_forked_amd.functional.nominal as FN
import torchmetrics_forked_amd.functional.pairwise as FP
import torchmetrics_forked_amd.nominal as NM
from tests.helpers.testers import RefFn, assert_allclose, run_class_metric_test


def _refmod(name):
    import importlib

    return importlib.import_module(f"torchmetrics.functional.{name}")


def _cat_data(g, n=200, k=4):
    p = torch.randint(0, k, (n,), generator=g)
    t = torch.where(torch.rand(n, generator=g) < 0.6, p, torch.randint(0, k, (n,), generator=g))
    return p, t


@pytest.mark.parametrize("fn", ["cramers_v", "tschuprows_t"])
@pytest.mark.parametrize("bias_correction", [True, False])
def test_nominal_bias(reference, fn, bias_correction):
    g = torch.Generator().manual_seed(0)
    p, t = _cat_data(g)
    assert_allclose(getattr(FN, fn)(p, t, bias_correction=bias_correction),
                    getattr(reference.functional.nominal, fn)(p, t, bias_correction=bias_correction), 1e-5)
    m = torch.randint(0, 3, (100, 4), generator=g)
    assert_allclose(getattr(FN, f"{fn}_matrix")(m, bias_correction=bias_correction),
                    getattr(reference.functional.nominal, f"{fn}_matrix")(m, bias_correction=bias_correction), 1e-5)


@pytest.mark.parametrize("fn", ["pearsons_contingency_coefficient", "theils_u"])
def test_nominal_other(reference, fn):
    g = torch.Generator().manual_seed(1)
    p, t = _cat_data(g)
    assert_allclose(getattr(FN, fn)(p, t), getattr(reference.functional.nominal, fn)(p, t), 1e-5)
    pf, tf = p.float(), t.float()
    pf[3] = float("nan")
    for strat in ("replace", "drop"):
        assert_allclose(getattr(FN, fn)(pf, tf, nan_strategy=strat), getattr(reference.functional.nominal, fn)(pf, tf, nan_strategy=strat), 1e-5)
    m = torch.randint(0, 3, (100, 4), generator=g)
    assert_allclose(getattr(FN, f"{fn}_matrix")(m), getattr(reference.functional.nominal, f"{fn}_matrix")(m), 1e-5)


def test_fleiss(reference):
    g = torch.Generator().manual_seed(2)
    counts = torch.multinomial(torch.ones(5), 10 * 50, replacement=True).reshape(50, 10)
    counts = torch.nn.functional.one_hot(counts, 5).sum(1)
    assert_allclose(FN.fleiss_kappa(counts), reference.functional.nominal.fleiss_kappa(counts), 1e-6)
    probs = torch.rand(50, 5, 7, generator=g)
    assert_allclose(FN.fleiss_kappa(probs, "probs"), reference.functional.nominal.fleiss_kappa(probs, "probs"), 1e-6)


@pytest.mark.parametrize("ddp", [False, True])
def test_nominal_modules(ddp):
    g = torch.Generator().manual_seed(3)
    P = torch.randint(0, 4, (4, 50), generator=g)
    T = torch.where(torch.rand(4, 50, generator=g) < 0.5, P, torch.randint(0, 4, (4, 50), generator=g))
    for cls, fn in ((NM.CramersV, "cramers_v"), (NM.TschuprowsT, "tschuprows_t"),
                    (NM.PearsonsContingencyCoefficient, "pearsons_contingency_coefficient"), (NM.TheilsU, "theils_u")):
        run_class_metric_test(ddp, P, T, cls, RefFn(fn, "nominal"), {"num_classes": 4}, atol=1e-5)


EXTRINSIC = ["mutual_info_score", "normalized_mutual_info_score", "adjusted_mutual_info_score", "rand_score",
             "adjusted_rand_score", "fowlkes_mallows_index", "homogeneity_score", "completeness_score", "v_measure_score"]


@pytest.mark.parametrize("fn", EXTRINSIC)
def test_clustering_extrinsic(reference, fn):
    g = torch.Generator().manual_seed(4)
    for k in (2, 5):
        p, t = _cat_data(g, 150, k)
        assert_allclose(getattr(FC, fn)(p, t), getattr(_refmod('clustering'), fn)(p, t), 1e-4)
    p = torch.randint(0, 3, (60,), generator=g) * 7 + 2  # non-contiguous ids
    t = torch.randint(0, 4, (60,), generator=g)
    assert_allclose(getattr(FC, fn)(p, t), getattr(_refmod('clustering'), fn)(p, t), 1e-4)


@pytest.mark.parametrize("method", ["min", "geometric", "arithmetic", "max"])
def test_clustering_average_methods(reference, method):
    g = torch.Generator().manual_seed(5)
    p, t = _cat_data(g, 120, 3)
    for fn in ("normalized_mutual_info_score", "adjusted_mutual_info_score"):
        assert_allclose(getattr(FC, fn)(p, t, method), getattr(_refmod('clustering'), fn)(p, t, method), 1e-4)


@pytest.mark.parametrize("fn", ["calinski_harabasz_score", "davies_bouldin_score", "dunn_index"])
def test_clustering_intrinsic(reference, fn):
    g = torch.Generator().manual_seed(6)
    data = torch.randn(100, 3, generator=g)
    labels = torch.randint(0, 4, (100,), generator=g)
    data = data + labels.unsqueeze(1).float() * 2
    assert_allclose(getattr(FC, fn)(data, labels), getattr(_refmod('clustering'), fn)(data, labels), 1e-4)


@pytest.mark.parametrize("ddp", [False, True])
def test_clustering_modules(ddp):
    g = torch.Generator().manual_seed(7)
    P = torch.randint(0, 3, (4, 40), generator=g)
    T = torch.randint(0, 3, (4, 40), generator=g)
    for name in ("MutualInfoScore", "RandScore", "AdjustedRandScore", "FowlkesMallowsIndex", "VMeasureScore",
                 "NormalizedMutualInfoScore", "AdjustedMutualInfoScore"):
        fn = {"MutualInfoScore": "mutual_info_score", "RandScore": "rand_score", "AdjustedRandScore": "adjusted_rand_score",
              "FowlkesMallowsIndex": "fowlkes_mallows_index", "VMeasureScore": "v_measure_score",
              "NormalizedMutualInfoScore": "normalized_mutual_info_score",
              "AdjustedMutualInfoScore": "adjusted_mutual_info_score"}[name]
        run_class_metric_test(ddp, P, T, getattr(CL, name), RefFn(fn, "clustering"), {}, atol=1e-4)
    D = torch.randn(4, 40, 3, generator=g)
    L = torch.randint(0, 3, (4, 40), generator=g)
    D = D + L.unsqueeze(-1).float()
    for name, fn in (("CalinskiHarabaszScore", "calinski_harabasz_score"), ("DaviesBouldinScore", "davies_bouldin_score"),
                     ("DunnIndex", "dunn_index")):
        run_class_metric_test(ddp, D, L, getattr(CL, name), RefFn(fn, "clustering"), {}, atol=1e-4)


@pytest.mark.parametrize("fn", ["pairwise_cosine_similarity", "pairwise_euclidean_distance", "pairwise_linear_similarity",
                                "pairwise_manhattan_distance", "pairwise_minkowski_distance"])
@pytest.mark.parametrize("reduction", [None, "mean", "sum"])
def test_pairwise(reference, fn, reduction):
    g = torch.Generator().manual_seed(8)
    x, y = torch.randn(30, 7, generator=g), torch.randn(20, 7, generator=g)
    R = getattr(reference.functional.pairwise, fn)
    M = getattr(FP, fn)
    kw = {"exponent": 3} if "minkowski" in fn else {}
    assert_allclose(M(x, y, reduction=reduction, **kw), R(x, y, reduction=reduction, **kw), 1e-4)
    assert_allclose(M(x, reduction=reduction, **kw), R(x, reduction=reduction, **kw), 1e-4)
    assert_allclose(M(x, y, zero_diagonal=True, **kw), R(x, y, zero_diagonal=True, **kw), 1e-4)
