"""Batched Hungarian assignment for PIT: host solver (tmx::linear_assignment) and the GPU wave solver
(tmx::linear_assignment_gpu) against brute force over all permutations, ties and non-finite entries included."""
from itertools import permutations

import pytest
import torch

from torchmetrics_forked_amd import ops

pytestmark = pytest.mark.skipif(not ops.load(), reason="native library not built")


def _brute(m, maximize):
    S = m.shape[-1]
    best = []
    for b in range(m.shape[0]):
        vals = [sum(float(m[b, i, p[i]]) for i in range(S)) for p in permutations(range(S))]
        best.append(max(vals) if maximize else min(vals))
    return torch.tensor(best, dtype=torch.float64)


def _score(m, perm):
    return torch.gather(m.double(), 2, perm[:, :, None].to(m.device)).sum((1, 2)).cpu()


def _problems(S, B=120, seed=0, ties=False):
    g = torch.Generator().manual_seed(seed + S)
    if ties:
        return torch.randint(-3, 4, (B, S, S), generator=g).double()
    return torch.randn(B, S, S, generator=g, dtype=torch.float64)


@pytest.mark.parametrize("S", [1, 2, 3, 4, 5, 6])
@pytest.mark.parametrize("maximize", [True, False])
@pytest.mark.parametrize("ties", [False, True])
def test_host_solver_is_optimal(S, maximize, ties):
    m = _problems(S, ties=ties)
    perm = torch.ops.tmx.linear_assignment(m, maximize)
    assert torch.equal(torch.sort(perm, dim=1).values, torch.arange(S).expand(m.shape[0], S))
    torch.testing.assert_close(_score(m, perm), _brute(m, maximize), rtol=0, atol=1e-9)


def test_host_solver_non_finite_entries_terminate():
    m = torch.randn(4, 5, 5, dtype=torch.float64)
    m[0, 1] = float("nan")
    m[1, :, 2] = float("inf")
    m[2] = float("-inf")
    m[3, 0, 0] = float("nan")
    perm = torch.ops.tmx.linear_assignment(m, True)
    assert torch.equal(torch.sort(perm, dim=1).values, torch.arange(5).expand(4, 5))


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
@pytest.mark.parametrize("S", [1, 2, 3, 4, 5, 8, 16, 33, 64])
@pytest.mark.parametrize("maximize", [True, False])
@pytest.mark.parametrize("ties", [False, True])
def test_gpu_solver_matches_host(S, maximize, ties):
    m = _problems(S, B=300, seed=7, ties=ties)
    host = torch.ops.tmx.linear_assignment(m, maximize)
    dev = torch.ops.tmx.linear_assignment_gpu(m.cuda(), maximize)
    assert torch.equal(dev.cpu(), host)  # same operations in the same order: the same assignment
    if S <= 6:
        torch.testing.assert_close(_score(m, dev.cpu()), _brute(m, maximize), rtol=0, atol=1e-9)


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
def test_gpu_solver_non_finite_and_pit():
    m = torch.randn(4, 5, 5, dtype=torch.float64)
    m[0, 1] = float("nan")
    m[1, :, 2] = float("inf")
    m[2] = float("-inf")
    dev = torch.ops.tmx.linear_assignment_gpu(m.cuda(), True).cpu()
    assert torch.equal(dev, torch.ops.tmx.linear_assignment(m, True))
    from torchmetrics_forked_amd.functional.audio import permutation_invariant_training, scale_invariant_signal_distortion_ratio

    g = torch.Generator().manual_seed(3)
    preds, target = torch.randn(16, 5, 800, generator=g), torch.randn(16, 5, 800, generator=g)
    a = permutation_invariant_training(preds, target, scale_invariant_signal_distortion_ratio, eval_func="max")
    b = permutation_invariant_training(preds.cuda(), target.cuda(), scale_invariant_signal_distortion_ratio, eval_func="max")
    assert torch.equal(a[1], b[1].cpu())
    torch.testing.assert_close(a[0], b[0].cpu(), rtol=1e-5, atol=1e-5)
