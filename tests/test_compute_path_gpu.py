"""compute()-path launches: ``tmx::curve_hist_scores`` equals ``curve_hist_reduce`` + ``curve_summary`` bit for bit
across repeated launches and on a side stream; ``tmx::gather_flags`` (written straight into mapped pinned
memory) returns every flag and clears the consumed ones."""
import pytest
import torch

from torchmetrics_forked_amd import ops
from torchmetrics_forked_amd.ops import classification as K

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_native(device):
    ops.require()


def _hist(C, seed):
    g = torch.Generator().manual_seed(seed)
    h = torch.zeros(C, 2, K.N_CODES, dtype=torch.long)
    lo = torch.randint(0, 8000, (C,), generator=g)
    for c in range(C):
        span = slice(int(lo[c]), int(lo[c]) + 3000)
        h[c, 0, span] = torch.randint(0, 50, (3000,), generator=g)
        h[c, 1, span] = torch.randint(0, 3, (3000,), generator=g) * (c % 7 != 3)  # some classes without positives
    rng = torch.stack([lo, lo + 2999], 1).int()
    return h.cuda(), rng.cuda()


@pytest.mark.parametrize("C", [1, 3, 257, 1000])
def test_fused_scores_match_two_launches(C):
    h, rng = _hist(C, C)
    sc_ref = torch.ops.tmx.curve_hist_reduce(h, rng)
    summ_ref = torch.ops.tmx.curve_summary(sc_ref)
    for _ in range(3):
        sc, summ = torch.ops.tmx.curve_hist_scores(h, rng)
        assert torch.equal(sc.view(torch.int64), sc_ref.view(torch.int64))  # bitwise: AP of a class without positives is NaN
        assert torch.equal(summ.view(torch.int64)[:8], summ_ref.view(torch.int64)[:8])
        assert torch.equal(summ[8:12].view(torch.float32), summ_ref[8:12].view(torch.float32))
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        sc2, summ2 = torch.ops.tmx.curve_hist_scores(h, rng)
    s.synchronize()
    assert torch.equal(sc2.view(torch.int64), sc_ref.view(torch.int64)) and torch.equal(summ2[:8].view(torch.int64), summ_ref[:8].view(torch.int64))


def test_gather_flags_into_pinned_memory():
    a = torch.tensor([0, 1, 0], dtype=torch.int32, device="cuda")
    b = torch.tensor([True], device="cuda")
    c = torch.tensor([2.0, 0.0], dtype=torch.float32, device="cuda")
    d = torch.tensor([5], dtype=torch.int64, device="cuda")
    out = torch.ops.tmx.gather_flags([a, b, c, d], [1, 0, 1, 0])
    assert not out.is_cuda and out.is_pinned()
    assert out.tolist() == [0, 1, 0, 1, 2, 0, 5]
    assert a.tolist() == [0, 0, 0] and c.tolist() == [0.0, 0.0]  # consumed
    assert b.tolist() == [True] and d.tolist() == [5]
    many = [torch.full((1,), i, dtype=torch.int32, device="cuda") for i in range(100)]  # more than one launch
    assert torch.ops.tmx.gather_flags(many, [0] * 100).tolist() == list(range(100))
