"""Mispredicted normalisation mode on the headline two-pass route (csrc/curve_hist_kernels.h ``class_hist_block``
refit): the row pass speculates softmax-vs-raw from the previous batch; when the guess is wrong the class pass
rebuilds its class's codes from the scores with the row pass's per-row softmax statistics instead of a FIXUP launch.
The histogram and confusion matrix of a mispredicted batch must be bit-identical to the same batch predicted correctly
(same GPU arithmetic), including ignored rows, NaN / inf rows, and fp16 / bf16 inputs; its code range must cover the
correct one (``_range_covers``)."""
import pytest
import torch

from torchmetrics_forked_amd import ops
from torchmetrics_forked_amd.ops import classification as K

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_native(device):
    ops.require()


def _batch(N, C, probs, dtype, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(N, C, generator=g) * 2
    if probs:
        x = x.softmax(1)
    x[5::97, min(3, C - 1)] = float("nan")
    x[11::131, C // 2] = float("inf")
    x[17::211] = float("-inf")
    x[23::53, 0] = x[23::53, min(2, C - 1)] = 0.75 if probs else 9.0
    t = torch.randint(0, C, (N,), generator=g)
    t[::19] = -1  # ignored rows
    return x.to(dtype).cuda(), t.cuda()


def _run(x, t, speculated):
    C = x.shape[1]
    hist = torch.zeros(C, 2, K.N_CODES, dtype=torch.long, device="cuda")
    cm = torch.zeros(C, C, dtype=torch.long, device="cuda")
    rng = torch.full((C, 2), -1, dtype=torch.int32, device="cuda")
    rng[:, 0] = K.N_CODES
    mode = torch.zeros(8, dtype=torch.int32, device="cuda")
    mode[0] = speculated
    K.curve_hist_update(x, t, hist, "multiclass", -1, cm, None, mode, rng)
    torch.cuda.synchronize()
    return hist, cm, rng, mode


@pytest.mark.parametrize("C", [10, 64, 250, 520, 1000])  # small-class route (C <= 256) and the tile route
@pytest.mark.parametrize("probs", [False, True])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_refit_matches_correct_prediction(C, probs, dtype):
    x, t = _batch(3001, C, probs, dtype, seed=C + int(probs))
    # the sprinkled NaN / inf make every batch a softmax batch (reference rule): mode 1 is the right guess
    good = _run(x, t, speculated=1)
    bad = _run(x, t, speculated=0)
    assert int(good[3][1]) == 0 and int(bad[3][0]) == 1  # rolled: the next batch speculates softmax
    assert torch.equal(good[0], bad[0])
    assert torch.equal(good[1], bad[1])
    _range_covers(bad[2], good[2], C)


def _range_covers(got, want, C):
    """The tile route's row pass books each positive (and widens its class's code range) before the class pass knows
    the speculation was wrong; the refit takes the histogram count back but a code range stays widened -- a bound,
    never narrower than the correct one (compute scans a few more empty bins).  The small-class route is exact."""
    if C <= 256:
        assert torch.equal(got, want)
        return
    occupied = want[:, 1] >= 0
    assert bool((got[occupied, 0] <= want[occupied, 0]).all()) and bool((got[occupied, 1] >= want[occupied, 1]).all())


@pytest.mark.parametrize("C", [10, 520, 1000])
def test_refit_probability_batch(C):
    """A clean probability batch (no witness) speculated as softmax: the refit keeps the raw scores' codes."""
    g = torch.Generator().manual_seed(7)
    x = torch.randn(4096, C, generator=g).softmax(1).bfloat16().cuda()
    t = torch.randint(0, C, (4096,), generator=g).cuda()
    t[::23] = -1
    good = _run(x, t, speculated=0)
    bad = _run(x, t, speculated=1)
    assert torch.equal(good[0], bad[0]) and torch.equal(good[1], bad[1])
    _range_covers(bad[2], good[2], C)
    assert int(bad[3][0]) == 0  # rolled back to raw scores for the next batch


@pytest.mark.parametrize("C", [16, 520])
def test_refit_rows_beyond_one_chunk(C):
    """> 65528 rows: the refit rewrites the whole class slice, the counting loop flushes per chunk as usual."""
    g = torch.Generator().manual_seed(11)
    N = 70_000
    x = (torch.randn(N, C, generator=g) * 3).bfloat16().cuda()
    t = torch.randint(0, C, (N,), generator=g).cuda()
    good = _run(x, t, speculated=1)
    bad = _run(x, t, speculated=0)
    assert torch.equal(good[0], bad[0])
    _range_covers(bad[2], good[2], C)
    assert good[0].sum().item() == N * C


def test_small_route_error_flag_with_mode_word():
    x, t = _batch(5000, 10, False, torch.bfloat16, seed=5)
    t = t.clamp(min=0)
    t[17] = 12
    hist = torch.zeros(10, 2, K.N_CODES, dtype=torch.long, device="cuda")
    mode = torch.zeros(8, dtype=torch.int32, device="cuda")
    err = torch.zeros(1, dtype=torch.int32, device="cuda")
    K.curve_hist_update(x, t, hist, "multiclass", None, None, err, mode, None)
    torch.cuda.synchronize()
    assert int(err) == 1


@pytest.mark.parametrize("N", [65536, 65544, 131072])
def test_u16_full_chunk_single_code_columns(N):
    """Tile route, whole 65536-row chunks: a class whose every code is one negative value would wrap its 16-bit LDS
    half (low-half and high-half bins), an all-positive identical column is exact modulo 2^32 -- the histogram must
    equal the host bincount in every case."""
    C = 520
    g = torch.Generator().manual_seed(N)
    x = torch.rand(N, C, generator=g) * 0.9 + 0.05  # probabilities: raw-score codes (bf16 bits)
    x[:, 3] = 1e-20  # code < 8192: low half of its LDS word
    x[:, 5] = 0.25  # code >= 8192: high half
    x[:, 7] = 0.125
    t = torch.full((N,), 7, dtype=torch.long)  # every row positive for class 7, negative for 3 and 5
    t[N // 2 :: 3] = torch.randint(8, C, (len(range(N // 2, N, 3)),), generator=g)
    xb = x.bfloat16()
    hist, _, _, mode = _run(xb.cuda(), t.cuda(), speculated=0)
    assert int(mode[0]) == 0
    codes = xb.view(torch.int16).long() & 0xFFFF
    for c in (3, 5, 7, 8, 519):
        pos = t == c
        ref_neg = torch.bincount(codes[~pos, c], minlength=K.N_CODES)
        ref_pos = torch.bincount(codes[pos, c], minlength=K.N_CODES)
        assert torch.equal(hist[c, 0].cpu(), ref_neg), c
        assert torch.equal(hist[c, 1].cpu(), ref_pos), c
    assert int(hist.sum()) == N * C
