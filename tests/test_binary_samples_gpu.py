"""GPU fp32 / fp64 binary curve samples (csrc/binary_samples.hip): the fused format pass (target value check, sigmoid
decision on device, copy) and the capped positive count, against plain torch (fp32 reference of the same op)."""
import pytest
import torch

import torchmetrics_forked_amd as tm
from torchmetrics_forked_amd import ops
from torchmetrics_forked_amd.ops import classification as K

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_native(device):
    ops.require()


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("n", [1, 7, 4096, 1_000_003])
def test_sigmoid_bit_identical_to_torch(dtype, n):
    g = torch.Generator(device="cuda").manual_seed(n)
    x = torch.randn(n, device="cuda", generator=g, dtype=dtype) * 12
    x[:: max(1, n // 5)] = 200.0  # saturating logits: ties at 1.0 must match torch exactly
    t = torch.randint(0, 2, (n,), device="cuda", generator=g)
    out = K.binary_samples_format(x, t, None)
    ref = torch.sigmoid(x) if not bool(((x >= 0) & (x <= 1)).all()) else x
    assert out.dtype == dtype and out.shape == (n,)
    assert torch.equal(out, ref)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_probabilities_pass_through_and_unaligned(dtype):
    g = torch.Generator(device="cuda").manual_seed(1)
    base = torch.rand(100_001, device="cuda", generator=g, dtype=dtype)
    x = base[1:]  # 4/8-byte offset: not 16-B aligned
    t = torch.randint(0, 2, (100_000,), device="cuda", generator=g)
    assert torch.equal(K.binary_samples_format(x, t, None), x)
    y = x.clone()
    y[-1] = float("nan")  # NaN trips the flag (reference: not all in [0, 1] -> sigmoid)
    out = K.binary_samples_format(y, t, None)
    torch.testing.assert_close(out, torch.sigmoid(y), rtol=0, atol=0, equal_nan=True)


@pytest.mark.parametrize("tdtype", [torch.int64, torch.int32, torch.uint8, torch.int8, torch.bool])
def test_target_check_flag(tdtype):
    n = 50_001
    x = torch.rand(n, device="cuda")
    t = torch.randint(0, 2, (n,), device="cuda").to(tdtype)
    err = torch.zeros(1, dtype=torch.int32, device="cuda")
    K.binary_samples_format(x, t, err)
    assert int(err) == 0
    if tdtype is not torch.bool:
        t2 = t.clone()
        t2[n - 1] = 2  # in the scalar tail of the vectorised check
        K.binary_samples_format(x, t2, err)
        assert int(err) == 1
        err.zero_()
        t3 = t.clone()
        t3[17] = 3
        K.binary_samples_format(x, t3, err)
        assert int(err) == 1


def test_count_exceeds():
    t = torch.zeros(3_000_000, dtype=torch.long, device="cuda")
    assert K.count_exceeds(t, 1, 8192) == 0
    t[:8192] = 1
    assert K.count_exceeds(t, 1, 8192) == 8192
    t[-1] = 1
    assert K.count_exceeds(t, 1, 8192) > 8192
    t.fill_(1)
    assert K.count_exceeds(t, 1, 8192) > 8192
    assert K.count_exceeds(t.bool(), 1, 10) > 10


@pytest.mark.parametrize("n, pos_frac", [(1000, 0.5), (200_000, 0.02), (3_000_001, 0.5)])
def test_binary_modules_fp32_match_cpu(n, pos_frac):
    g = torch.Generator().manual_seed(n)
    x = torch.randn(n, generator=g) * 3
    t = (torch.rand(n, generator=g) < pos_frac).long()
    for cls in (tm.BinaryAUROC, tm.BinaryAveragePrecision):
        cpu, gpu = cls(), cls().cuda()
        for sl in (slice(0, n // 3), slice(n // 3, n)):
            cpu.update(x[sl], t[sl])
            gpu.update(x[sl].cuda(), t[sl].cuda())
        torch.testing.assert_close(gpu.compute().cpu().double(), cpu.compute().double(), rtol=1e-6, atol=1e-7)
    # single update: the compute reads the stored batch without a concatenation copy
    m = tm.BinaryAUROC().cuda()
    m.update(x.cuda(), t.cuda())
    ref = tm.BinaryAUROC()
    ref.update(x, t)
    torch.testing.assert_close(m.compute().cpu().double(), ref.compute().double(), rtol=1e-6, atol=1e-7)
    assert m.preds[0].shape == (n,) and bool(((m.preds[0] >= 0) & (m.preds[0] <= 1)).all())


def test_binary_invalid_target_raises_at_compute():
    m = tm.BinaryAUROC().cuda()
    x = torch.rand(1000, device="cuda")
    t = torch.randint(0, 2, (1000,), device="cuda")
    t[5] = 2
    m.update(x, t)
    with pytest.raises(RuntimeError):
        m.compute()
