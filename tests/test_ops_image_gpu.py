"""gfx950 fused SSIM window kernel vs the grouped-conv PyTorch formulation (CPU) of the reference algorithm."""
import pytest
import torch

from torchmetrics_forked_amd import ops

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_native(device):
    ops.require()


@pytest.mark.parametrize("shape", [(2, 3, 64, 64), (1, 1, 11, 11), (3, 2, 300, 517), (1, 3, 1024, 1024)])
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
