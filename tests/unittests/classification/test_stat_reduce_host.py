"""``stat_reduce_host`` (csrc/host_classification.cpp): the one-call CPU reduction of (tp, fp, tn, fn) equals the ATen
chain of ``functional/classification/_stat_family.py`` it replaces -- bit for bit for elementwise / micro averages,
within one float32 ulp for macro / weighted (class sums accumulated in double there)."""
import pytest
import torch

from torchmetrics_forked_amd.functional.classification import _stat_family as fam


def _states(shape, seed, zero_frac=0.2):
    g = torch.Generator().manual_seed(seed)
    st = [torch.randint(0, 50, shape, generator=g) for _ in range(4)]
    mask = torch.rand(shape, generator=g) < zero_frac  # classes with no tp / fp / fn at all
    for t in (st[0], st[1], st[3]):
        t[mask] = 0
    return st


REDUCERS = {
    "accuracy": fam._accuracy_reduce,
    "precision": lambda *a, **k: fam._precision_recall_reduce("precision", *a, **k),
    "recall": lambda *a, **k: fam._precision_recall_reduce("recall", *a, **k),
    "f1": lambda *a, **k: fam._fbeta_reduce(*a[:4], 1.0, *a[4:], **k),
    "f0.5": lambda *a, **k: fam._fbeta_reduce(*a[:4], 0.5, *a[4:], **k),
    "f2": lambda *a, **k: fam._fbeta_reduce(*a[:4], 2.0, *a[4:], **k),
    "specificity": fam._specificity_reduce,
    "hamming": fam._hamming_distance_reduce,
}


@pytest.mark.parametrize("name", list(REDUCERS))
@pytest.mark.parametrize("average", ["binary", "micro", "macro", "weighted", "none"])
@pytest.mark.parametrize("multidim", ["global", "samplewise"])
@pytest.mark.parametrize("multilabel", [False, True])
def test_stat_reduce_host_matches_aten_chain(monkeypatch, name, average, multidim, multilabel):
    from torchmetrics_forked_amd import ops

    if not ops.load():
        pytest.skip("native library not built")
    shape = (7,) if multidim == "global" else (4, 7)
    if average == "binary":
        shape = () if multidim == "global" else (9,)
    tp, fp, tn, fn = _states(shape, hash((name, average, multidim, multilabel)) % 1000)
    red = REDUCERS[name]
    native = red(tp.clone(), fp.clone(), tn.clone(), fn.clone(), average=average, multidim_average=multidim, multilabel=multilabel)
    monkeypatch.setattr(fam, "_host_reduce", lambda *a, **k: None)
    ref = red(tp.clone(), fp.clone(), tn.clone(), fn.clone(), average=average, multidim_average=multidim, multilabel=multilabel)
    assert native.dtype == ref.dtype and native.shape == ref.shape
    if average in ("macro", "weighted"):
        torch.testing.assert_close(native, ref, rtol=2.4e-7, atol=0)
    else:
        assert torch.equal(native, ref)


def test_stat_reduce_host_micro_scalar_states(monkeypatch):
    from torchmetrics_forked_amd import ops

    if not ops.load():
        pytest.skip("native library not built")
    tp, fp, tn, fn = (torch.tensor(v) for v in (5, 3, 40, 0))
    native = fam._accuracy_reduce(tp, fp, tn, fn, average="micro")
    monkeypatch.setattr(fam, "_host_reduce", lambda *a, **k: None)
    assert torch.equal(native, fam._accuracy_reduce(tp, fp, tn, fn, average="micro"))
