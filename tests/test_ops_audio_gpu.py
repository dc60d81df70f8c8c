"""gfx950 Levinson Toeplitz solver (SDR) vs the dense fp64 solve, and GPU audio metrics vs CPU."""
import pytest
import torch

from torchmetrics_forked_amd import ops

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_native(device):
    ops.require()


@pytest.mark.parametrize("n,L", [(1, 1), (3, 7), (64, 512), (8, 2048), (300, 128)])
def test_toeplitz_solve_kernel(n, L):
    from torchmetrics_forked_amd.functional.audio.sdr import _compute_autocorr_crosscorr, _symmetric_toeplitz

    g = torch.Generator().manual_seed(L)
    t = torch.randn(n, 4 * L + 100, generator=g, dtype=torch.float64)
    p = t + 0.3 * torch.randn(n, 4 * L + 100, generator=g, dtype=torch.float64)
    r0, b = _compute_autocorr_crosscorr(t, p, L)
    sol = torch.ops.tmx.toeplitz_solve(r0.cuda(), b.cuda()).cpu()
    ref = torch.linalg.solve(_symmetric_toeplitz(r0), b)
    torch.testing.assert_close(sol, ref, atol=1e-8, rtol=1e-6)
    torch.testing.assert_close(torch.ops.tmx.toeplitz_solve(r0, b), ref, atol=1e-8, rtol=1e-6)


@pytest.mark.parametrize("name", ["signal_distortion_ratio", "scale_invariant_signal_distortion_ratio", "signal_noise_ratio"])
def test_audio_gpu_matches_cpu(name):
    import torchmetrics_forked_amd.functional.audio as F

    g = torch.Generator().manual_seed(0)
    t = torch.randn(4, 2, 8000, generator=g)
    p = t + 0.2 * torch.randn(4, 2, 8000, generator=g)
    torch.testing.assert_close(getattr(F, name)(p.cuda(), t.cuda()).cpu(), getattr(F, name)(p, t), atol=1e-4, rtol=1e-5)


def test_pit_gpu_hungarian():
    import torchmetrics_forked_amd.functional.audio as F

    g = torch.Generator().manual_seed(1)
    t = torch.randn(8, 5, 400, generator=g)
    p = t[:, torch.randperm(5, generator=g)] + 0.1 * torch.randn(8, 5, 400, generator=g)
    a = F.permutation_invariant_training(p.cuda(), t.cuda(), F.scale_invariant_signal_distortion_ratio)
    b = F.permutation_invariant_training(p, t, F.scale_invariant_signal_distortion_ratio)
    torch.testing.assert_close(a[0].cpu(), b[0], atol=1e-4, rtol=1e-5)
    assert torch.equal(a[1].cpu(), b[1])


@pytest.mark.parametrize("C,T,K", [(1, 10, 3), (184, 16000, 3), (1472, 4000, 3), (7, 999, 5)])
def test_iir_filter_kernel(C, T, K):
    g = torch.Generator().manual_seed(C + T)
    x = torch.randn(C, T, generator=g, dtype=torch.float64)
    b = torch.randn(C, K, generator=g, dtype=torch.float64)
    a = torch.zeros(C, K, dtype=torch.float64)
    a[:, 0] = 2.0
    a[:, 1] = -0.9  # stable poles
    torch.testing.assert_close(torch.ops.tmx.iir_filter(x.cuda(), b.cuda(), a.cuda()).cpu(), torch.ops.tmx.iir_filter(x, b, a),
                               atol=1e-10, rtol=1e-10)


def test_srmr_and_stoi_gpu_match_cpu():
    import torchmetrics_forked_amd.functional.audio as F

    g = torch.Generator().manual_seed(2)
    t = torch.arange(16000) / 16000
    x = (0.3 * torch.sin(2 * torch.pi * 300 * t) * (1 + torch.sin(2 * torch.pi * 4 * t)))[None].repeat(2, 1)
    x = x + 0.05 * torch.randn(2, 16000, generator=g)
    torch.testing.assert_close(F.speech_reverberation_modulation_energy_ratio(x.cuda().double(), 16000).cpu(),
                               F.speech_reverberation_modulation_energy_ratio(x.double(), 16000), atol=1e-8, rtol=1e-8)
    y = x + 0.2 * torch.randn(2, 16000, generator=g)
    torch.testing.assert_close(F.short_time_objective_intelligibility(y.cuda(), x.cuda(), 16000), 
                               F.short_time_objective_intelligibility(y, x, 16000), atol=1e-8, rtol=1e-8)
