"""Fused MFMA pairwise GEMM forms (``csrc/pairwise.hip`` ``pairwise_gemm``: linear / cosine / euclidean with the
epilogue in the kernel) against plain PyTorch fp64 references of the same op, and the public functional API on the GPU
against the reference composition (reference ``functional/pairwise/{linear,cosine,euclidean}.py``)."""
import pytest
import torch

from torchmetrics_forked_amd import ops

pytestmark = pytest.mark.gpu

SHAPES = [((1, 1), (1, 1)), ((70, 33), (130, 33)), ((257, 100), (64, 100)), ((64, 64), (64, 64)), ((300, 7), (129, 7)),
          ((513, 256), (1000, 256)), ((65, 1000), (66, 1000))]


@pytest.fixture(scope="module", autouse=True)
def _need_native(device):
    ops.require()


def _ref(mode, x, y, zero_diag):
    """fp64 reference of the op; for euclidean the reference's own rounding steps (fp64 sum, cast, zero, root)."""
    xd, yd = x.double(), y.double()
    if mode == 0:
        out = (xd @ yd.T).to(x.dtype)
    elif mode == 1:
        out = ((xd / xd.norm(dim=1, keepdim=True)) @ (yd / yd.norm(dim=1, keepdim=True)).T).to(x.dtype)
    else:
        d = ((xd * xd).sum(1, keepdim=True) + (yd * yd).sum(1) - 2 * xd @ yd.T).to(x.dtype)
        if zero_diag:
            d.fill_diagonal_(0)
        return d.sqrt()
    if zero_diag:
        out.fill_diagonal_(0)
    return out


def _tol(mode, dtype, D):
    if dtype == torch.float64:
        return 1e-10, 1e-10
    if dtype == torch.float32:
        return (2e-5, 2e-5 * max(1, D) ** 0.5) if mode == 0 else (1e-5, 1e-5)
    return 1e-2, (1e-2 * max(1, D) ** 0.5 if mode == 0 else 1e-2)  # one 16-bit rounding of the result


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64, torch.bfloat16, torch.float16])
def test_pairwise_gemm_vs_fp64(shape, mode, dtype):
    g = torch.Generator().manual_seed(sum(shape[0]) * 7 + mode)
    x = torch.randn(*shape[0], generator=g).to(dtype).cuda()
    y = torch.randn(*shape[1], generator=g).to(dtype).cuda()
    for zd in (False, True):
        out = torch.ops.tmx.pairwise_gemm(x, y, mode, zd)
        assert out.dtype == dtype and out.shape == (shape[0][0], shape[1][0])
        ref = _ref(mode, x, y, zd)
        rtol, atol = _tol(mode, dtype, shape[0][1])
        torch.testing.assert_close(out.double(), ref.double(), rtol=rtol, atol=atol, equal_nan=True)


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_pairwise_gemm_unaligned_and_strided(mode):
    """A view whose storage offset breaks 16-B alignment (scalar-load path) and a transposed (non-contiguous) input."""
    g = torch.Generator().manual_seed(5)
    base = torch.randn(200 * 64 + 1, generator=g).cuda()
    x = base[1:].view(200, 64)  # 4-B offset: D % 8 == 0 but not 16-B aligned
    y = torch.randn(64, 150, generator=g).cuda().T  # [150, 64], not contiguous
    out = torch.ops.tmx.pairwise_gemm(x, y, mode, False)
    torch.testing.assert_close(out.double(), _ref(mode, x, y, False).double(), rtol=2e-5, atol=2e-4)


def test_functional_api_takes_the_fused_kernel_and_matches_the_composition():
    import torchmetrics_forked_amd.functional.pairwise as FP
    from torchmetrics_forked_amd.functional.pairwise import helpers

    g = torch.Generator().manual_seed(11)
    x, y = torch.randn(300, 48, generator=g).cuda(), torch.randn(200, 48, generator=g).cuda()
    cases = ((FP.pairwise_linear_similarity, 0), (FP.pairwise_cosine_similarity, 1), (FP.pairwise_euclidean_distance, 2))
    for fn, mode in cases:  # (300 x 200 x 48: the kernel's side of the measured routing)
        for args, zd in (((x, y), None), ((x,), None), ((x, y), True), ((x,), False)):
            if mode == 2 and len(args) == 1 and zd is False:
                continue  # |x|^2 + |x|^2 - 2 x.x rounds to +-eps on the diagonal: sqrt of a negative is NaN in both
            got = fn(*args, zero_diagonal=zd)
            yy = args[1] if len(args) > 1 else args[0]
            want_zd = (len(args) == 1) if zd is None else zd
            assert torch.equal(got, torch.ops.tmx.pairwise_gemm(args[0], yy, mode, want_zd)), (fn.__name__, zd)
            # the ATen composition the reference runs (native route disabled for this call)
            helpers._FUSED = False
            try:
                comp = fn(*args, zero_diagonal=zd)
            finally:
                helpers._FUSED = True
            torch.testing.assert_close(got, comp, rtol=1e-5, atol=1e-4)
        for red in ("mean", "sum"):
            torch.testing.assert_close(fn(x, y, reduction=red), getattr(torch.ops.tmx.pairwise_gemm(x, y, mode, False), red)(-1))


def test_autograd_and_mixed_dtypes_take_the_aten_path():
    import torchmetrics_forked_amd.functional.pairwise as FP

    x = torch.randn(20, 8, device="cuda", requires_grad=True)
    y = torch.randn(10, 8, device="cuda")
    d = FP.pairwise_euclidean_distance(x, y)
    d.sum().backward()
    assert x.grad is not None and torch.isfinite(x.grad).all()
    mixed = FP.pairwise_euclidean_distance(x.detach(), y.double())
    assert mixed.dtype == torch.float32
    torch.testing.assert_close(mixed, FP.pairwise_euclidean_distance(x.detach(), y), rtol=1e-6, atol=1e-6)


def test_routing_sends_deep_or_large_products_to_the_library():
    from torchmetrics_forked_amd.functional.pairwise import helpers

    assert helpers._fused_wins("euclidean", torch.float32, 8192, 8192, 1024)
    assert not helpers._fused_wins("euclidean", torch.float32, 4096, 4096, 2048)
    assert helpers._fused_wins("linear", torch.float32, 1000, 1000, 128)
    assert helpers._fused_wins("cosine", torch.bfloat16, 4096, 4096, 512)  # 16-bit MFMA tiles
    assert not helpers._fused_wins("cosine", torch.bfloat16, 8192, 8192, 64)
    assert not helpers._fused_wins("linear", torch.bfloat16, 1000, 1000, 1024)
    assert not helpers._fused_wins("linear", torch.float64, 1000, 1000, 128)
    assert helpers._fused_wins("cosine", torch.float64, 1000, 1000, 128)


@pytest.mark.parametrize("D", [64, 100])
@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_pairwise_gemm_16bit_mfma_tiles(D, mode, dtype):
    """>= 256 128 x 128 output tiles of 16-bit linear / cosine take the v_mfma_f32_16x16x32 kernel (D = 100: the
    element-wise staging path)."""
    g = torch.Generator().manual_seed(D + mode)
    x = torch.randn(2048, D, generator=g).to(dtype).cuda()
    y = torch.randn(2100, D, generator=g).to(dtype).cuda()
    for zd in (False, True):
        out = torch.ops.tmx.pairwise_gemm(x, y, mode, zd)
        torch.testing.assert_close(out.double(), _ref(mode, x, y, zd).double(), rtol=1e-2, atol=1e-2 * (D ** 0.5 if mode == 0 else 1))
