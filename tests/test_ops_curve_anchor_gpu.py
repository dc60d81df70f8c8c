"""Positive-anchored exact AUROC / AP for fp32 scores (csrc/curve_anchor.hip) vs the sort-based fp64
formulation of the same quantities (``_curve_engine.samples_scores``), on tie-heavy inputs."""
import pytest
import torch

from torchmetrics_forked_amd import ops
from torchmetrics_forked_amd.functional.classification import _curve_engine as eng

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_native(device):
    ops.require()


def _quantised(shape, levels, g):
    x = torch.rand(*shape, generator=g)
    if levels == -1:  # log-uniform over ~26 binades: coarse anchor buckets holding many keys each
        return torch.exp(-18 * x)
    return (x * levels).floor() / levels if levels else x


@pytest.mark.parametrize("n,c,levels", [(5000, 7, 16), (4096, 1000, 0), (3001, 33, 64), (257, 5, 2), (65536, 100, 0),
                                          (28000, 8, -1)])
def test_anchored_multiclass_matches_sorted(n, c, levels):
    g = torch.Generator().manual_seed(n + c)
    preds = _quantised((n, c), levels, g).softmax(1) if levels == 0 else _quantised((n, c), levels, g)
    target = torch.randint(0, c, (n,), generator=g)
    target[target == c - 1] = 0  # class c-1 has no positives
    got = eng.anchored_scores(preds.cuda(), target.cuda(), "multiclass", c, None)
    assert got is not None
    labels = torch.nn.functional.one_hot(target, c).bool()
    ref = torch.stack(eng.samples_scores(preds.double(), labels), 1)
    torch.testing.assert_close(got.cpu()[:, 2:], ref[:, 2:], atol=0, rtol=0)
    torch.testing.assert_close(got.cpu()[:, :2], ref[:, :2], atol=1e-12, rtol=0, equal_nan=True)


@pytest.mark.parametrize("n,c,levels", [(2000, 6, 8), (777, 3, 0)])
def test_anchored_multilabel_and_binary_match_sorted(n, c, levels):
    g = torch.Generator().manual_seed(3 * n + c)
    preds = _quantised((n, c), levels, g)
    target = (torch.rand(n, c, generator=g) < 0.2).long()
    target[:, 0] = 1  # label 0: no negatives
    got = eng.anchored_scores(preds.cuda(), target.cuda(), "multilabel", c, None)
    ref = torch.stack(eng.samples_scores(preds.double(), target == 1), 1)
    torch.testing.assert_close(got.cpu(), ref, atol=1e-12, rtol=0, equal_nan=True)
    gb = eng.anchored_scores(preds[:, 1].contiguous().cuda(), target[:, 1].cuda(), "binary", 1, None)
    rb = torch.stack(eng.samples_scores(preds[:, 1].double(), target[:, 1] == 1), 1)
    torch.testing.assert_close(gb.cpu(), rb, atol=1e-12, rtol=0, equal_nan=True)


def test_anchored_falls_back_for_dense_positives():
    g = torch.Generator().manual_seed(0)
    preds = torch.rand(40000, generator=g)
    target = (torch.rand(40000, generator=g) < 0.5).long()
    assert eng.anchored_scores(preds.cuda(), target.cuda(), "binary", 1, None) is None


@pytest.mark.parametrize("c", [50, 52])
@pytest.mark.parametrize("average", ["macro", "weighted", "none"])
def test_multiclass_auroc_ap_fp32_module_gpu_vs_cpu(average, c):
    """c = 52: class-major update + anchored compute; c = 50: row-major fallback (C % 4 != 0)."""
    import torchmetrics_forked_amd as tm

    g = torch.Generator().manual_seed(11)
    n = 6000
    preds = _quantised((n, c), 32, g)
    target = torch.randint(0, c, (n,), generator=g)
    for cls in (tm.MulticlassAUROC, tm.MulticlassAveragePrecision):
        gpu = cls(num_classes=c, average=average).cuda()
        cpu = cls(num_classes=c, average=average)
        for i in range(3):
            sl = slice(i * 2000, (i + 1) * 2000)
            gpu.update(preds[sl].cuda(), target[sl].cuda())
            cpu.update(preds[sl], target[sl])
        torch.testing.assert_close(gpu.compute().cpu(), cpu.compute(), atol=1e-6, rtol=0)


@pytest.mark.parametrize("c", [12, 1000, 36, 4])
def test_softmax_colmajor_matches_aten(c):
    from torchmetrics_forked_amd.ops import classification as cls_ops

    g = torch.Generator().manual_seed(c)
    x = torch.randn(1003, c, generator=g).cuda()
    got = cls_ops.softmax_colmajor(x)
    torch.testing.assert_close(got.t(), x.softmax(1), atol=2e-7, rtol=1e-6)
    probs = x.softmax(1)  # already in [0, 1]: identity
    assert torch.equal(cls_ops.softmax_colmajor(probs).t(), probs)


def test_multiclass_fp32_state_is_class_major_and_checkpoint_compatible():
    import torchmetrics_forked_amd as tm

    g = torch.Generator().manual_seed(2)
    x = torch.randn(517, 20, generator=g)
    t = torch.randint(0, 20, (517,), generator=g)
    m = tm.MulticlassAUROC(num_classes=20).cuda()
    m.update(x.cuda(), t.cuda())
    st = m.preds[0]
    assert st.shape == (517, 20) and st.t().is_contiguous()
    torch.testing.assert_close(st.cpu(), x.softmax(1), atol=2e-7, rtol=1e-6)
    cpu = tm.MulticlassAUROC(num_classes=20)
    cpu.update(x, t)
    torch.testing.assert_close(m.compute().cpu(), cpu.compute(), atol=1e-6, rtol=0)
    # the state dict round-trips into a CPU metric (reference layout: rows [N, C])
    m2 = tm.MulticlassAUROC(num_classes=20)
    m2.persistent(True)
    m.persistent(True)
    m2.load_state_dict({k: (v.cpu() if isinstance(v, torch.Tensor) else [e.cpu() for e in v]) for k, v in m.state_dict().items()})
    torch.testing.assert_close(m2.compute(), cpu.compute(), atol=1e-6, rtol=0)


def test_multiclass_fp32_target_range_checked_in_kernel():
    import torchmetrics_forked_amd as tm

    m = tm.MulticlassAUROC(num_classes=5).cuda()
    m.update(torch.randn(10, 5).cuda(), torch.tensor([0, 1, 2, 3, 4, 5, 0, 1, 2, 3]).cuda())
    with pytest.raises(RuntimeError):
        m.compute()
    ok = tm.MulticlassAUROC(num_classes=5, ignore_index=7).cuda()
    ok.update(torch.randn(10, 5).cuda(), torch.tensor([0, 1, 2, 3, 4, 7, 0, 1, 2, 3]).cuda())
    assert torch.isfinite(ok.compute())
