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
    assert helpers._fused_wins("linear", torch.float32, 4096, 4096, 512)  # fp32 x3 route (>= 256 128 x 128 tiles)
    assert helpers._fused_wins("cosine", torch.float32, 10000, 10000, 2048)
    assert not helpers._fused_wins("linear", torch.float32, 1000, 1000, 2048)
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


def _x3_err(out, x, y, mode):
    """Max |out - fp64 ref| and the same for ATen's fp32 GEMM of the op (the precision the reference delivers)."""
    ref = _ref(mode, x, y, False).double()
    if mode == 0:
        aten = x @ y.T
    else:
        aten = (x / x.norm(dim=1, keepdim=True)) @ (y / y.norm(dim=1, keepdim=True)).T
    return (out.double() - ref).abs().max().item(), (aten.double() - ref).abs().max().item()


@pytest.mark.parametrize("D", [33, 100, 512, 2048])
@pytest.mark.parametrize("mode", [0, 1])
def test_pairwise_gemm_fp32_split_f16_route(D, mode):
    """fp32 with >= 256 128 x 128 tiles runs on f16 matrix cores as hi·hi + hi·lo + lo·hi of a per-row scaled
    two-plane split (csrc/pairwise.hip x3): its error against fp64 stays within ATen's own fp32 GEMM error."""
    g = torch.Generator().manual_seed(D * 3 + mode)
    x = torch.randn(2053, D, generator=g).cuda()
    y = torch.randn(2100, D, generator=g).cuda()
    x[7] *= 1e-30  # tiny and huge rows: per-row power-of-two scales keep both planes in f16 range
    y[9] *= 3e28
    x[11] = 0.0
    for zd in (False, True):
        out = torch.ops.tmx.pairwise_gemm(x, y, mode, zd)
        ref = _ref(mode, x, y, zd).double()
        if mode == 1:  # the zero row is NaN in both (0 / 0)
            assert torch.isnan(out[11]).all() == torch.isnan(ref[11]).all()
            keep = torch.ones(x.shape[0], dtype=torch.bool, device=x.device)
            keep[11] = False
            out, ref = out[keep], ref[keep]
        assert not torch.isnan(out).any()
        if mode == 0:  # scale-aware: compare each output against |x_i| |y_j|
            scale = x.double().norm(dim=1, keepdim=True) @ y.double().norm(dim=1, keepdim=True).T
            if zd:
                scale.fill_diagonal_(1.0)
            assert ((out.double() - ref).abs() / scale.clamp_min(1e-300)).max().item() < 4e-7 * max(1, D) ** 0.5
        else:
            assert (out.double() - ref).abs().max().item() < 2e-6
    e_x3, e_aten = _x3_err(torch.ops.tmx.pairwise_gemm(x[12:], y[:2000], mode, False), x[12:], y[:2000], mode)
    assert e_x3 <= 4.0 * e_aten, (e_x3, e_aten)


def test_pairwise_gemm_fp32_split_nonfinite_falls_back_on_device():
    """An inf in a linear operand: the x3 route flags it and the exact fp32 kernel reruns on device (inf, not the
    NaN of inf - inf in the split)."""
    g = torch.Generator().manual_seed(3)
    x = torch.randn(2048, 64, generator=g).cuda()
    y = torch.randn(2048, 64, generator=g).cuda()
    x[5, 3] = float("inf")
    out = torch.ops.tmx.pairwise_gemm(x, y, 0, False)
    torch.testing.assert_close(out.double(), _ref(0, x, y, False).double(), rtol=2e-5, atol=2e-4, equal_nan=True)
    assert torch.isinf(out[5]).any()


@pytest.mark.parametrize("n,d", [(2100, 2048), (2500, 100)])
def test_abs_cos_rowmax_fp32_split_route(n, d):
    """MiFID's row max |cos| on the x3 route against fp64 and against the exact fp32 MFMA kernel (env switch)."""
    import os

    g = torch.Generator().manual_seed(n + d)
    a = torch.randn(n, d, generator=g).cuda()
    b = torch.randn(n - 37, d, generator=g).cuda()
    b[:50] = a[:50] * 0.5 + 1e-3 * b[:50]  # near duplicates: |cos| ~ 1
    got = torch.ops.tmx.pairwise_abs_cos_rowmax(a, b)
    ad, bd = a.double(), b.double()
    ref = ((ad / ad.norm(dim=1, keepdim=True)) @ (bd / bd.norm(dim=1, keepdim=True)).T).abs().max(dim=1).values
    assert (got.double() - ref).abs().max().item() < 1e-6
    os.environ["TMX_PAIRWISE_X3_OFF"] = "1"
    try:
        exact = torch.ops.tmx.pairwise_abs_cos_rowmax(a, b)
    finally:
        del os.environ["TMX_PAIRWISE_X3_OFF"]
    # both within fp32 GEMM error of fp64 (the exact fp32 kernel's own error at d = 2048 is ~1e-6)
    e_exact = (exact.double() - ref).abs().max().item()
    assert (got.double() - ref).abs().max().item() <= max(2 * e_exact, 1e-6)
    assert abs((1 - got).double().mean().item() - (1 - ref).mean().item()) < 2e-7
