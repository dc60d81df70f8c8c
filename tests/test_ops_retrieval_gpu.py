"""gfx950 segmented retrieval kernel (csrc/retrieval.hip, one wave per query) vs the eager CPU engine of the same
functions: every module and functional metric, with top-k / adaptive-k, tie-heavy scores (tie-averaged nDCG),
graded relevance, queries with no positives, and queries longer than a wave."""
import importlib

import pytest
import torch

import torchmetrics_forked_amd.retrieval as M
from torchmetrics_forked_amd import ops

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_native(device):
    ops.require()


FN = [
    ("retrieval_average_precision", {}), ("retrieval_average_precision", {"top_k": 3}),
    ("retrieval_reciprocal_rank", {}), ("retrieval_reciprocal_rank", {"top_k": 70}),
    ("retrieval_precision", {}), ("retrieval_precision", {"top_k": 4}), ("retrieval_precision", {"top_k": 300, "adaptive_k": True}),
    ("retrieval_precision", {"top_k": 300}), ("retrieval_recall", {"top_k": 65}), ("retrieval_fall_out", {"top_k": 5}),
    ("retrieval_hit_rate", {"top_k": 2}), ("retrieval_r_precision", {}), ("retrieval_normalized_dcg", {}),
    ("retrieval_normalized_dcg", {"top_k": 3}), ("retrieval_normalized_dcg", {"top_k": 100}),
]


@pytest.mark.parametrize("fn,kw", FN)
@pytest.mark.parametrize("n", [1, 17, 64, 200])
@pytest.mark.parametrize("ties", [False, True])
def test_functional_gpu_vs_cpu(fn, kw, n, ties):
    f = getattr(importlib.import_module("torchmetrics_forked_amd.functional.retrieval"), fn)
    g = torch.Generator().manual_seed(n + 7 * ties)
    p = torch.rand(n, generator=g)
    if ties:
        p = (p * 5).round() / 5
    t = torch.randint(0, 4 if "dcg" in fn else 2, (n,), generator=g)
    cpu = f(p, t, **kw)
    gpu = f(p.cuda(), t.cuda(), **kw).cpu()
    torch.testing.assert_close(gpu, cpu, rtol=1e-5, atol=1e-6)


MODULES = [
    ("RetrievalMAP", {}), ("RetrievalMAP", {"top_k": 2}), ("RetrievalMRR", {}), ("RetrievalPrecision", {"top_k": 3}),
    ("RetrievalPrecision", {"top_k": 8, "adaptive_k": True}), ("RetrievalRecall", {"top_k": 3}), ("RetrievalFallOut", {"top_k": 3}),
    ("RetrievalHitRate", {"top_k": 2}), ("RetrievalRPrecision", {}), ("RetrievalNormalizedDCG", {}),
    ("RetrievalNormalizedDCG", {"top_k": 2}),
]


@pytest.mark.parametrize("action", ["neg", "pos", "skip"])
@pytest.mark.parametrize("cls,kw", MODULES)
def test_modules_gpu_vs_cpu(cls, kw, action):
    g = torch.Generator().manual_seed(3)
    mc, mg = getattr(M, cls)(empty_target_action=action, **kw), getattr(M, cls)(empty_target_action=action, **kw).cuda()
    for _ in range(3):
        n = 5000
        idx = torch.randint(0, 300, (n,), generator=g)
        p = (torch.rand(n, generator=g) * 20).round() / 20
        t = torch.randint(0, 4 if "DCG" in cls else 2, (n,), generator=g)
        t[idx % 17 == 0] = 0  # queries without positives
        mc.update(p, t, indexes=idx)
        mg.update(p.cuda(), t.cuda(), indexes=idx.cuda())
    torch.testing.assert_close(mg.compute().cpu(), mc.compute(), rtol=1e-5, atol=1e-6)


def test_segments_stats_table():
    from torchmetrics_forked_amd.functional.retrieval._grouped import Grouped

    p = torch.tensor([0.9, 0.5, 0.5, 0.1, 0.7, 0.7]).cuda()
    t = torch.tensor([0, 1, 1, 0, 1, 0]).cuda()
    idx = torch.tensor([0, 0, 0, 0, 1, 1]).cuda()
    st = Grouped(p, t, idx).stats(2).cpu()
    # query 0 sorted: 0.9(0) 0.5(1) 0.5(1) 0.1(0): rel 2, neg 2, rel@2 1, neg@2 1, AP num 1/2, first 1, rel@R(2) 1
    assert st[0, :7].tolist() == [2.0, 2.0, 1.0, 1.0, 0.5, 1.0, 1.0]
    assert st[1, 0].item() == 1.0 and st[1, 9].item() == 2.0
