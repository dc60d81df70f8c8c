"""K6 for fp32 / fp64 at any size: the hand-written segmented radix sort + fused tie-group scan (csrc/radix.hip)
against the vectorised CPU implementation of the same exact definitions (``_curve_engine.samples_scores`` /
``samples_curve_points*``, i.e. the reference's ``_binary_clf_curve`` semantics)."""
import pytest
import torch

from torchmetrics_forked_amd import ops
from torchmetrics_forked_amd.functional.classification import _curve_engine as eng
from torchmetrics_forked_amd.ops import classification as K

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_native(device):
    ops.require()


def _scores(n, S, dtype, ties, gen):
    x = torch.rand(n, S, generator=gen, dtype=torch.float64)
    if ties:  # heavy ties: 50 distinct values, so tie groups span many 4096-key tiles
        x = (x * 50).floor() / 50
    x[::97] = -x[::97]  # negatives and -0.0 / +0.0 mixes
    x[5::1001] = 0.0
    x[6::1001] = -0.0
    return x.to(dtype)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("ties", [False, True])
@pytest.mark.parametrize("n", [1, 4095, 4097, 100_003, 4_300_003])  # the last: > 1024 tiles (two chunks of the tile-sum scan)
def test_sorted_binary_matches_cpu(dtype, ties, n):
    gen = torch.Generator().manual_seed(n)
    p = _scores(n, 1, dtype, ties, gen).reshape(-1)
    t = torch.randint(0, 2, (n,), generator=gen)
    got = eng.sorted_scores(p.cuda(), t.cuda(), "binary", None).cpu()
    ref = torch.stack(eng.samples_scores(p, t == 1), 1)
    torch.testing.assert_close(got, ref, rtol=1e-12, atol=1e-12, equal_nan=True)
    pts = eng.sorted_curve_points(p.cuda(), t.cuda(), "binary", None)[0]
    rf, rt, rthr = eng.samples_curve_points(p, t == 1)
    assert torch.equal(pts[0].cpu(), rf.float()) and torch.equal(pts[1].cpu(), rt.float())
    assert torch.equal(pts[2].cpu(), rthr)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("ties", [False, True])
def test_sorted_multiclass_matches_cpu(dtype, ties):
    gen = torch.Generator().manual_seed(3)
    n, C = 60_000, 7
    p = _scores(n, C, dtype, ties, gen)
    t = torch.randint(0, C, (n,), generator=gen)
    got = eng.sorted_scores(p.cuda(), t.cuda(), "multiclass", None).cpu()
    labels = torch.nn.functional.one_hot(t, C).bool()
    ref = torch.stack(eng.samples_scores(p, labels), 1)
    torch.testing.assert_close(got, ref, rtol=1e-12, atol=1e-12, equal_nan=True)
    pts = eng.sorted_curve_points(p.cuda(), t.cuda(), "multiclass", None)
    refp = eng.samples_curve_points_columns(p, labels)
    for (a, b, c), (x, y, z) in zip(pts, refp):
        assert torch.equal(a.cpu(), x.float()) and torch.equal(b.cpu(), y.float()) and torch.equal(c.cpu(), z)


def test_sorted_multilabel_ignore_matches_cpu():
    gen = torch.Generator().manual_seed(4)
    n, L = 30_000, 5
    p = _scores(n, L, torch.float32, True, gen)
    t = torch.randint(0, 2, (n, L), generator=gen)
    t[::7, 1] = -1
    t[::3, 4] = -1
    got = eng.sorted_scores(p.cuda(), t.cuda(), "multilabel", -1).cpu()
    ref = torch.stack(eng.samples_scores(p, t == 1, t != -1), 1)
    torch.testing.assert_close(got, ref, rtol=1e-12, atol=1e-12, equal_nan=True)
    pts = eng.sorted_curve_points(p.cuda(), t.cuda(), "multilabel", -1)
    for i, (a, b, c) in enumerate(pts):
        keep = t[:, i] != -1
        x, y, z = eng.samples_curve_points(p[keep, i], t[keep, i] == 1)
        assert torch.equal(a.cpu(), x.float()) and torch.equal(b.cpu(), y.float()) and torch.equal(c.cpu(), z), i


def test_modules_fp32_many_positives_use_radix(monkeypatch):
    """MulticlassAUROC / AveragePrecision / ROC fp32 with > ANCHOR_MAX_POS positives per class: GPU == CPU."""
    import torchmetrics_forked_amd as tm

    called = []
    orig = K.curve_sorted
    monkeypatch.setattr(K, "curve_sorted", lambda *a, **k: called.append(1) or orig(*a, **k))
    gen = torch.Generator().manual_seed(9)
    C, n = 3, 30_000  # ~10k positives per class
    x = torch.randn(n, C, generator=gen).softmax(1)  # probabilities: both devices store identical scores
    t = torch.randint(0, C, (n,), generator=gen)
    res = {}
    for dev in ("cuda", "cpu"):
        auroc = tm.MulticlassAUROC(num_classes=C, average=None).to(dev)
        ap = tm.MulticlassAveragePrecision(num_classes=C, average=None).to(dev)
        roc = tm.MulticlassROC(num_classes=C).to(dev)
        for m in (auroc, ap, roc):
            m.update(x.to(dev), t.to(dev))
        res[dev] = (auroc.compute().cpu(), ap.compute().cpu(), [r.cpu() for r in roc.compute()[0]])
    assert called
    torch.testing.assert_close(res["cuda"][0], res["cpu"][0], rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(res["cuda"][1], res["cpu"][1], rtol=1e-6, atol=1e-7)
    for a, b in zip(res["cuda"][2], res["cpu"][2]):
        torch.testing.assert_close(a, b)
