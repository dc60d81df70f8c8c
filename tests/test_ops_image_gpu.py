"""gfx950 fused SSIM window kernel vs the grouped-conv PyTorch formulation (CPU) of the reference algorithm."""
import pytest
import torch

from torchmetrics_forked_amd import ops

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_native(device):
    ops.require()


@pytest.mark.parametrize("shape", [(2, 3, 64, 64), (1, 1, 11, 11), (3, 2, 300, 517), (2, 3, 300, 520), (1, 3, 1024, 1024)])
@pytest.mark.parametrize("kw", [{}, {"sigma": 0.8}, {"sigma": 2.0}, {"gaussian_kernel": False, "kernel_size": 7},
                                {"data_range": 1.0}, {"return_contrast_sensitivity": True}])
def test_ssim_native_vs_cpu(shape, kw):
    from torchmetrics_forked_amd.functional.image import structural_similarity_index_measure as ssim

    if kw.get("sigma", 1.5) == 2.0 and min(shape[-2:]) < 15:
        pytest.skip("window larger than image")
    g = torch.Generator().manual_seed(sum(shape))
    t = torch.rand(*shape, generator=g)
    p = (t + 0.1 * torch.randn(*shape, generator=g)).clamp(0, 1)
    a = ssim(p.cuda(), t.cuda(), reduction="none", **kw)
    b = ssim(p, t, reduction="none", **kw)
    if isinstance(a, tuple):
        for x, y in zip(a, b):
            assert torch.allclose(x.cpu(), y, atol=2e-5), (x, y)
    else:
        assert torch.allclose(a.cpu(), b, atol=2e-5), (a, b)


@pytest.mark.parametrize("ks", [3, 5, 9, 13, 15])
def test_ssim_v2_window_sizes(ks):
    """The 16-B-staged packed-fp32 kernel (fp32, W % 4 == 0) at every window size, strips not multiple of the block."""
    from torchmetrics_forked_amd.functional.image import structural_similarity_index_measure as ssim

    g = torch.Generator().manual_seed(ks)
    t = torch.rand(2, 2, 277, 388, generator=g)
    p = (t + 0.1 * torch.randn(2, 2, 277, 388, generator=g)).clamp(0, 1)
    kw = {"gaussian_kernel": False, "kernel_size": ks, "data_range": 1.0, "reduction": "none"}
    assert torch.allclose(ssim(p.cuda(), t.cuda(), **kw).cpu(), ssim(p, t, **kw), atol=2e-5)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_ssim_native_half(dtype):
    from torchmetrics_forked_amd.functional.image import structural_similarity_index_measure as ssim

    g = torch.Generator().manual_seed(3)
    t = torch.rand(2, 3, 128, 128, generator=g)
    p = (t + 0.1 * torch.randn(2, 3, 128, 128, generator=g)).clamp(0, 1)
    a = ssim(p.to(dtype).cuda(), t.to(dtype).cuda(), data_range=1.0, reduction="none").float().cpu()
    b = ssim(p.to(dtype).float(), t.to(dtype).float(), data_range=1.0, reduction="none")
    assert torch.allclose(a, b, atol=1e-2)


def test_ms_ssim_and_psnr_gpu():
    from torchmetrics_forked_amd.functional.image import (
        multiscale_structural_similarity_index_measure as msssim,
        peak_signal_noise_ratio as psnr,
    )

    g = torch.Generator().manual_seed(4)
    t = torch.rand(2, 3, 256, 256, generator=g)
    p = (t + 0.1 * torch.randn(2, 3, 256, 256, generator=g)).clamp(0, 1)
    assert torch.allclose(msssim(p.cuda(), t.cuda()).cpu(), msssim(p, t), atol=1e-5)
    assert torch.allclose(psnr(p.cuda(), t.cuda()).cpu(), psnr(p, t), atol=1e-4)


@pytest.mark.parametrize("net", ["alex", "vgg", "squeeze"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_lpips_fused_head_vs_eager(net, dtype):
    from torchmetrics_forked_amd.functional.image.lpips import _NoTrainLpips, _normalize_tensor

    torch.manual_seed(0)
    lp = _NoTrainLpips(net=net).cuda()
    a = (torch.rand(3, 3, 96, 80, device="cuda") * 2 - 1)
    b = (torch.rand(3, 3, 96, 80, device="cuda") * 2 - 1)
    with torch.no_grad():
        feats0, feats1 = lp.net(lp.scaling_layer(a)), lp.net(lp.scaling_layer(b))
        for f0, f1, lin in zip(feats0, feats1, lp.lins):
            f0, f1 = f0.to(dtype), f1.to(dtype)
            w = lin.model[-1].weight.reshape(-1)
            fused = torch.ops.tmx.lpips_head(f0, f1, w).float()
            eager = (((_normalize_tensor(f0.float()) - _normalize_tensor(f1.float())) ** 2) * w.view(1, -1, 1, 1)).sum(1).mean((1, 2))
            tol = 1e-5 if dtype == torch.float32 else 1e-4
            assert torch.allclose(fused, eager.double().float(), rtol=1e-4, atol=tol), (fused, eager)
            # channels_last feature maps: the NHWC kernels read them in place (fp32 with C % 4 == 0: four threads per
            # pixel, another summation order)
            cl = torch.ops.tmx.lpips_head(f0.contiguous(memory_format=torch.channels_last),
                                          f1.contiguous(memory_format=torch.channels_last), w).float()
            assert torch.allclose(cl, fused, rtol=1e-5, atol=1e-7), (cl, fused)
        val = lp(a, b)
    assert val.shape == (3, 1, 1, 1) and torch.isfinite(val).all()


def test_fid_gpu_vs_cpu():
    from torchmetrics_forked_amd.image.generative import _compute_fid

    g = torch.Generator().manual_seed(0)
    a, b = torch.randn(600, 256, generator=g, dtype=torch.float64), torch.randn(500, 256, generator=g, dtype=torch.float64)
    s1, s2 = torch.cov(a.T), torch.cov(b.T)
    m1, m2 = a.mean(0), b.mean(0)
    gpu = _compute_fid(m1.cuda(), s1.cuda(), m2.cuda(), s2.cuda()).cpu()
    cpu = _compute_fid(m1, s1, m2, s2)
    assert torch.allclose(gpu, cpu, rtol=1e-8)


@pytest.mark.parametrize("shape", [(2, 3, 300, 520), (1, 2, 1024, 1024), (3, 1, 64, 68)])
def test_fused_ssim_psnr_collection(shape):
    """MetricCollection{SSIM, PSNR}: the SSIM kernel also accumulates the squared error (ops/fused.py image_pair plan);
    results equal the separately updated metrics."""
    from torchmetrics_forked_amd import MetricCollection
    from torchmetrics_forked_amd.image import PeakSignalNoiseRatio, StructuralSimilarityIndexMeasure

    g = torch.Generator().manual_seed(sum(shape))
    t = torch.rand(*shape, generator=g)
    p = (t + 0.1 * torch.randn(*shape, generator=g)).clamp(0, 1)
    coll = MetricCollection({"ssim": StructuralSimilarityIndexMeasure(data_range=1.0),
                             "psnr": PeakSignalNoiseRatio(data_range=1.0)}).cuda()
    sep = [StructuralSimilarityIndexMeasure(data_range=1.0).cuda(), PeakSignalNoiseRatio(data_range=1.0).cuda()]
    for _ in range(2):
        coll.update(p.cuda(), t.cuda())
        for m in sep:
            m.update(p.cuda(), t.cuda())
    assert coll._fused_plans and type(coll._fused_plans[0]).__name__ == "_ImagePairPlan"
    out = coll.compute()
    assert torch.allclose(out["ssim"].cpu(), sep[0].compute().cpu(), atol=1e-6)
    assert torch.allclose(out["psnr"].cpu(), sep[1].compute().cpu(), atol=1e-4)
    assert int(coll["psnr"].total) == int(sep[1].total)


@pytest.mark.parametrize("shape", [(256, 2048), (37, 100), (5, 64), (1, 3), (200, 130)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64, torch.bfloat16])
def test_fid_gram_update_vs_fp64(shape, dtype):
    """Fused FID moments (``fid_gram_update``: upper tiles mirrored, feature sums on the diagonal tiles) against the
    fp64 torch reference ``x.double().T @ x.double()`` / ``sum``, accumulated over two updates."""
    g = torch.Generator().manual_seed(sum(shape))
    x = torch.randn(*shape, generator=g).to(dtype).cuda()
    F = shape[1]
    gram = torch.zeros(F, F, dtype=torch.float64, device="cuda")
    colsum = torch.zeros(F, dtype=torch.float64, device="cuda")
    for _ in range(2):
        torch.ops.tmx.fid_gram_update(x, gram, colsum)
    xd = x.double()
    torch.testing.assert_close(gram, 2 * xd.T @ xd, rtol=1e-12, atol=1e-10)
    torch.testing.assert_close(colsum, 2 * xd.sum(0), rtol=1e-12, atol=1e-10)
    assert torch.equal(gram, gram.T)


def test_fid_metric_fused_moments_match_cpu():
    """FrechetInceptionDistance with a small feature extractor: GPU (fused moments) vs CPU (double + sum + addmm)."""
    from torchmetrics_forked_amd.image import FrechetInceptionDistance

    class Feat(torch.nn.Module):
        def __init__(self):
            super().__init__()
            g = torch.Generator().manual_seed(0)
            self.register_buffer("w", torch.randn(3 * 4, 320, generator=g))

        def forward(self, x):
            x = torch.nn.functional.adaptive_avg_pool2d(x.float(), 2).flatten(1)
            return torch.tanh(x / 128.0 - 1.0) @ self.w

    g = torch.Generator().manual_seed(1)
    real = torch.randint(0, 256, (40, 3, 32, 32), generator=g, dtype=torch.uint8)
    fake = torch.randint(0, 200, (40, 3, 32, 32), generator=g, dtype=torch.uint8)
    from torchmetrics_forked_amd.image.generative import _fused_moments

    assert _fused_moments(torch.zeros(2, 320, device="cuda"), torch.zeros(320, 320, dtype=torch.float64, device="cuda"),
                          torch.zeros(320, dtype=torch.float64, device="cuda"))
    vals = []
    for dev in ("cuda", "cpu"):
        m = FrechetInceptionDistance(feature=Feat()).to(dev)
        for i in range(2):
            m.update(real[20 * i:20 * (i + 1)].to(dev), real=True)
            m.update(fake[20 * i:20 * (i + 1)].to(dev), real=False)
        vals.append(m.compute().cpu())
    torch.testing.assert_close(vals[0], vals[1], rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize(("n", "m", "d", "degree"), [(300, 100, 64, 3), (150, 150, 37, 2), (90, 65, 130, 1)])
def test_kid_poly_sums_vs_torch(dtype, n, m, d, degree):
    """Fused KID subset sums (``kid_poly_sums``) against the reference's poly_kernel / maximum_mean_discrepancy terms on
    the gathered subsets, in fp64."""
    g = torch.Generator().manual_seed(n + m + d)
    real = torch.randn(n, d, generator=g).to(dtype).cuda()
    fake = (torch.randn(n + 7, d, generator=g) + 0.3).to(dtype).cuda()
    ir, jf = torch.randperm(n, generator=g)[:m], torch.randperm(n + 7, generator=g)[:m]
    gamma, coef = 1.0 / d, 1.0
    sums = torch.ops.tmx.kid_poly_sums(real, fake, ir, jf, degree, gamma, coef)
    a, b = real.double()[ir.cuda()], fake.double()[jf.cuda()]
    k = lambda x, y: (x @ y.T * gamma + coef) ** degree  # noqa: E731
    kxx, kyy, kxy = k(a, a), k(b, b), k(a, b)
    ref = torch.stack([kxx.sum() - kxx.diag().sum(), kyy.sum() - kyy.diag().sum(), kxy.sum()])
    tol = 1e-10 if dtype == torch.float64 else 2e-5
    torch.testing.assert_close(sums, ref, rtol=tol, atol=tol * m * m)
    # several subsets in one launch: row s equals the single-subset call on subset s
    ir2 = torch.stack([ir, torch.randperm(n, generator=g)[:m]])
    jf2 = torch.stack([jf, torch.randperm(n + 7, generator=g)[:m]])
    many = torch.ops.tmx.kid_poly_sums(real, fake, ir2, jf2, degree, gamma, coef)
    assert many.shape == (2, 3)
    torch.testing.assert_close(many[0], sums, rtol=1e-12, atol=0)
    torch.testing.assert_close(many[1], torch.ops.tmx.kid_poly_sums(real, fake, ir2[1], jf2[1], degree, gamma, coef), rtol=1e-12, atol=0)
    with pytest.raises(RuntimeError, match="out of range"):
        torch.ops.tmx.kid_poly_sums(real, fake, torch.tensor([0, n]), torch.tensor([0, 1]), degree, gamma, coef)


@pytest.mark.parametrize(("m", "d", "degree"), [(1000, 2048, 3), (300, 257, 2)])
def test_kid_poly_sums_fp32_split_route(m, d, degree):
    """fp32 features of Inception depth take the f16-split matrix-core route (csrc/pairwise.hip kid_poly_x3_kernel:
    features split once, subset rows gathered into the shared x3 tile core); the three sums against fp64."""
    g = torch.Generator().manual_seed(m + d)
    real = torch.rand(m + 50, d, generator=g).cuda()
    fake = (torch.rand(m + 20, d, generator=g) * 1.1).cuda()
    ir, jf = torch.randperm(m + 50, generator=g)[:m], torch.randperm(m + 20, generator=g)[:m]
    gamma, coef = 1.0 / d, 1.0
    sums = torch.ops.tmx.kid_poly_sums(real, fake, ir, jf, degree, gamma, coef)
    a, b = real.double()[ir.cuda()], fake.double()[jf.cuda()]
    k = lambda x, y: (x @ y.T * gamma + coef) ** degree  # noqa: E731
    kxx, kyy, kxy = k(a, a), k(b, b), k(a, b)
    ref = torch.stack([kxx.sum() - kxx.diag().sum(), kyy.sum() - kyy.diag().sum(), kxy.sum()])
    torch.testing.assert_close(sums, ref, rtol=2e-6, atol=0)
    # the MMD the metric forms from them (reference kid.py maximum_mean_discrepancy) to ~1e-6 of its scale
    mmd = lambda s: s[0] / (m * (m - 1)) + s[1] / (m * (m - 1)) - 2 * s[2] / (m * m)  # noqa: E731
    assert abs(float(mmd(sums)) - float(mmd(ref))) < 1e-5 * float(ref[2] / (m * m))


def test_kid_metric_fused_matches_cpu():
    """KernelInceptionDistance compute on the GPU (fused subset sums) vs the CPU reference path, same randperm draws."""
    from torchmetrics_forked_amd.image import KernelInceptionDistance

    class Feat(torch.nn.Module):
        def __init__(self):
            super().__init__()
            g = torch.Generator().manual_seed(0)
            self.register_buffer("w", torch.randn(3 * 4, 70, generator=g))

        def forward(self, x):
            x = torch.nn.functional.adaptive_avg_pool2d(x.float(), 2).flatten(1)
            return torch.tanh(x / 128.0 - 1.0) @ self.w

    g = torch.Generator().manual_seed(1)
    real = torch.randint(0, 256, (120, 3, 16, 16), generator=g, dtype=torch.uint8)
    fake = torch.randint(0, 200, (110, 3, 16, 16), generator=g, dtype=torch.uint8)
    out = []
    for dev in ("cuda", "cpu"):
        m = KernelInceptionDistance(feature=Feat(), subsets=5, subset_size=100).to(dev)
        m.update(real.to(dev), real=True)
        m.update(fake.to(dev), real=False)
        torch.manual_seed(123)
        out.append([v.cpu() for v in m.compute()])
    torch.testing.assert_close(out[0][0], out[1][0], rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(out[0][1], out[1][1], rtol=1e-3, atol=1e-5)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64, torch.bfloat16])
@pytest.mark.parametrize(("n", "m", "d"), [(300, 200, 64), (70, 130, 33), (1, 5, 8), (257, 64, 100)])
def test_pairwise_abs_cos_rowmax_vs_torch(dtype, n, m, d):
    """MiFID's memorization term: row maxima of |cos| from the fused kernel vs the normalise / matmul / abs / max
    composition in fp64."""
    g = torch.Generator().manual_seed(n + m + d)
    x = torch.randn(n, d, generator=g).to(dtype).cuda()
    y = torch.randn(m, d, generator=g).to(dtype).cuda()
    got = torch.ops.tmx.pairwise_abs_cos_rowmax(x, y)
    xd, yd = x.double(), y.double()
    ref = ((xd / xd.norm(dim=1, keepdim=True)) @ (yd / yd.norm(dim=1, keepdim=True)).T).abs().max(dim=1).values
    tol = 1e-12 if dtype == torch.float64 else 2e-6
    torch.testing.assert_close(got.double(), ref, rtol=tol, atol=tol)


def test_mifid_cosine_distance_fused_matches_cpu():
    from torchmetrics_forked_amd.image.generative import _compute_cosine_distance

    g = torch.Generator().manual_seed(3)
    a = torch.randn(500, 96, generator=g)
    b = a[:400] + 0.05 * torch.randn(400, 96, generator=g)  # near-duplicates: a small memorization distance
    a[7] = 0.0  # a zero-sum row is dropped on both paths
    for eps in (0.1, 0.5):
        gpu = _compute_cosine_distance(a.cuda(), b.cuda(), eps).cpu()
        cpu = _compute_cosine_distance(a, b, eps)
        torch.testing.assert_close(gpu, cpu, rtol=1e-5, atol=1e-6)


def _ssim_raw(p, t, ks, consts, sse=True):
    w = torch.exp(-((torch.arange(ks, dtype=torch.float32) - (ks - 1) / 2) ** 2) / (2 * 1.5**2))
    w = (w / w.sum()).cuda()
    return torch.ops.tmx.ssim_sums(p, t, w, w, consts.cuda(), sse)


@pytest.mark.parametrize("shape", [(5, 257, 300), (3, 129, 1020), (2, 64, 64), (4, 1024, 1024), (1, 40, 2052)])
@pytest.mark.parametrize("ks", [3, 7, 11, 15])
@pytest.mark.parametrize("rng", [1.0, 255.0])
def test_ssim_mfma_vs_fp32_kernel(shape, ks, rng):
    """Round 6: the matrix-core SSIM kernel (fp16-split banded products, consts = c1, c2, data range) against the fp32
    VALU kernel (consts = c1, c2) on the same planes: per-plane mean SSIM / CS within 1e-6, SSE to fp64 summation order."""
    g = torch.Generator(device="cuda").manual_seed(sum(shape) + ks)
    t = torch.rand(*shape, device="cuda", generator=g) * rng
    p = (t + 0.1 * rng * torch.randn(*shape, device="cuda", generator=g)).clamp(0, rng)
    if rng == 255.0:
        p, t = p.round(), t.round()
    c = torch.tensor([(0.01 * rng) ** 2, (0.03 * rng) ** 2, rng])
    fast = _ssim_raw(p, t, ks, c)
    ref = _ssim_raw(p, t, ks, c[:2])
    nv = (shape[1] - ks + 1) * (shape[2] - ks + 1)
    torch.testing.assert_close(fast[:2] / nv, ref[:2] / nv, rtol=0, atol=1e-6)
    torch.testing.assert_close(fast[2], ref[2], rtol=1e-8, atol=0)  # fp64 sums of the same fp32 squares, another tile order


@pytest.mark.parametrize("bad", ["range", "nan", "inf"])
def test_ssim_mfma_falls_back_on_device(bad):
    """Data outside the kernel's fp16 operand range (here 10x the stated data range), NaN or inf: the fallback launch of
    the fp32 kernel runs on the device (no host synchronisation) and its sums are returned, bit for bit."""
    g = torch.Generator(device="cuda").manual_seed(5)
    t = torch.rand(3, 100, 128, device="cuda", generator=g)
    p = t.clone()
    if bad == "range":
        p = p * 10
    else:
        p[1, 50, 60] = float("nan") if bad == "nan" else float("inf")
    c = torch.tensor([1e-4, 9e-4, 1.0])
    fast = _ssim_raw(p, t, 11, c)
    ref = _ssim_raw(p, t, 11, c[:2])
    torch.testing.assert_close(fast, ref, rtol=0, atol=0, equal_nan=True)
