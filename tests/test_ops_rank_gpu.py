"""gfx950 rank kernels (csrc/rank.hip) vs the eager CPU path: Spearman's tie-averaged ranks and Kendall's
inversion count, on tie-heavy and tie-free data (exact: ranks are half-integers, counts are integers)."""
import pytest
import torch

import torchmetrics_forked_amd as tm
import torchmetrics_forked_amd.functional as F
from torchmetrics_forked_amd import ops

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_native(device):
    ops.require()


@pytest.mark.parametrize("n", [1, 2, 7, 1000, 1024, 1025, 100_000])
@pytest.mark.parametrize("ties", [False, True])
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_rank_average_vs_cpu(n, ties, dtype):
    from torchmetrics_forked_amd.functional.regression.spearman import _rank_data

    g = torch.Generator().manual_seed(n)
    x = (torch.randint(0, max(2, n // 10), (n,), generator=g).to(dtype) if ties else torch.randn(n, generator=g, dtype=dtype))
    assert torch.equal(_rank_data(x.cuda()).cpu(), _rank_data(x))


@pytest.mark.parametrize("n", [2, 3, 1023, 1024, 1025, 4096, 70_001])
@pytest.mark.parametrize("ties", [False, True])
def test_count_inversions_vs_cpu(n, ties):
    from torchmetrics_forked_amd.functional.regression import kendall as K

    g = torch.Generator().manual_seed(n + ties)
    y = torch.randint(0, 50, (n,), generator=g).double() if ties else torch.randn(n, generator=g, dtype=torch.float64)
    got = int(torch.ops.tmx.count_inversions(y.cuda()))
    assert got == int(K._count_inversions(y))
    if n <= 2000:  # brute force
        assert got == int((y[:, None] > y[None, :]).triu(1).sum())


@pytest.mark.parametrize("variant", ["a", "b", "c"])
@pytest.mark.parametrize("outputs", [1, 3])
def test_kendall_spearman_gpu_vs_cpu(variant, outputs):
    g = torch.Generator().manual_seed(outputs)
    shape = (5000, outputs) if outputs > 1 else (5000,)
    p = torch.randint(0, 30, shape, generator=g).float()
    t = p + torch.randn(shape, generator=g)
    cpu = F.kendall_rank_corrcoef(p, t, variant=variant)
    gpu = F.kendall_rank_corrcoef(p.cuda(), t.cuda(), variant=variant).cpu()
    torch.testing.assert_close(gpu, cpu, rtol=1e-6, atol=1e-7)
    cpu = F.spearman_corrcoef(p, t)
    gpu = F.spearman_corrcoef(p.cuda(), t.cuda()).cpu()
    torch.testing.assert_close(gpu, cpu, rtol=1e-6, atol=1e-7)
    m = tm.SpearmanCorrCoef(num_outputs=outputs).cuda()
    m.update(p.cuda(), t.cuda())
    torch.testing.assert_close(m.compute().cpu(), cpu, rtol=1e-6, atol=1e-7)
