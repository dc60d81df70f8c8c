"""Collection-level fusion (ops/fused.py + csrc/fused.hip): a MetricCollection of multiclass metrics that share the
scores is updated by one pass over [N, C] (+ confmat_fold), and must give exactly the states / values of the same
metrics updated one by one."""
import pytest
import torch

import torchmetrics_forked_amd as tm
from torchmetrics_forked_amd import ops

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_native(device):
    ops.require()


def _members(C, ii=None, curve=True):
    m = {
        "cm": tm.MulticlassConfusionMatrix(num_classes=C, ignore_index=ii),
        "acc": tm.MulticlassAccuracy(num_classes=C, ignore_index=ii),
        "acc_micro": tm.MulticlassAccuracy(num_classes=C, average="micro", ignore_index=ii),
        "f1": tm.MulticlassF1Score(num_classes=C, ignore_index=ii),
        "prec_w": tm.MulticlassPrecision(num_classes=C, average="weighted", ignore_index=ii),
        "rec_none": tm.MulticlassRecall(num_classes=C, average="none", ignore_index=ii),
        "spec": tm.MulticlassSpecificity(num_classes=C, ignore_index=ii),
        "stat": tm.MulticlassStatScores(num_classes=C, average="micro", ignore_index=ii),
    }
    if curve:
        m["auroc"] = tm.MulticlassAUROC(num_classes=C, ignore_index=ii)
    return m


@pytest.mark.parametrize("C,dtype,curve,ii", [(1000, torch.bfloat16, True, None), (64, torch.float16, True, 3),
                                              (100, torch.float32, False, None), (37, torch.bfloat16, False, 0)])
def test_fused_collection_matches_individual(C, dtype, curve, ii):
    g = torch.Generator(device="cuda").manual_seed(C)
    batches = [(torch.randn(3000, C, device="cuda", generator=g).to(dtype), torch.randint(0, C, (3000,), device="cuda", generator=g))
               for _ in range(3)]
    coll = tm.MetricCollection(_members(C, ii, curve)).cuda()
    solo = {k: v.cuda() for k, v in _members(C, ii, curve).items()}
    for p, t in batches:
        coll.update(p, t)
        for m in solo.values():
            m.update(p, t)
    assert coll._fused_plans and len(coll._fused_plans[0].names) == len(solo)
    got = coll.compute()
    for k, m in solo.items():
        torch.testing.assert_close(got[k], m.compute(), atol=0, rtol=0, msg=k)


def test_fused_collection_forward_matches_individual():
    C = 50
    g = torch.Generator(device="cuda").manual_seed(1)
    coll = tm.MetricCollection(_members(C)).cuda()
    solo = {k: v.cuda() for k, v in _members(C).items()}
    for _ in range(3):
        p = torch.randn(2000, C, device="cuda", generator=g).to(torch.bfloat16)
        t = torch.randint(0, C, (2000,), device="cuda", generator=g)
        out = coll(p, t)
        for k, m in solo.items():
            torch.testing.assert_close(out[k], m(p, t), atol=0, rtol=0, msg=k)
    got = coll.compute()
    for k, m in solo.items():
        torch.testing.assert_close(got[k], m.compute(), atol=0, rtol=0, msg=k)


def test_fused_collection_target_range_error_deferred():
    C = 16
    coll = tm.MetricCollection(_members(C, curve=False)).cuda()
    t = torch.randint(0, C, (100,), device="cuda")
    t[7] = C + 3
    coll.update(torch.randn(100, C, device="cuda"), t)
    with pytest.raises(RuntimeError):
        coll.compute()
