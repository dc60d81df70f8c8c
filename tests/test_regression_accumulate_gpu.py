"""In-place sum-state updates of MSE / MAE on the GPU (csrc/regression.hip ``regression_accumulate``): one map-reduce
launch plus one fold launch update the states; values must match the CPU eager path (fp64 reference sums)."""
import pytest
import torch

import torchmetrics_forked_amd as tm
from torchmetrics_forked_amd import ops

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_native(device):
    ops.require()


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("cls, kw", [(tm.MeanSquaredError, {}), (tm.MeanSquaredError, {"squared": False}),
                                     (tm.MeanSquaredError, {"num_outputs": 3}), (tm.MeanAbsoluteError, {})])
def test_accumulate_matches_cpu(dtype, cls, kw):
    g = torch.Generator().manual_seed(0)
    shape = (10_001, 3) if kw.get("num_outputs") == 3 else (10_001,)
    gpu, cpu = cls(**kw).cuda(), cls(**kw)
    for _ in range(4):
        p = torch.randn(*shape, generator=g, dtype=dtype)
        t = torch.randn(*shape, generator=g, dtype=dtype)
        gpu.update(p.cuda(), t.cuda())
        cpu.update(p, t)
    torch.testing.assert_close(gpu.compute().cpu(), cpu.compute(), rtol=1e-6, atol=1e-7)
    assert int(gpu.total) == int(cpu.total)
    gpu.reset()
    gpu.update(p.cuda(), t.cuda())
    cpu.reset()
    cpu.update(p, t)
    torch.testing.assert_close(gpu.compute().cpu(), cpu.compute(), rtol=1e-6, atol=1e-7)


def test_accumulate_float64_state_and_autograd_fallback():
    g = torch.Generator().manual_seed(1)
    p = torch.randn(5000, generator=g).cuda()
    t = torch.randn(5000, generator=g).cuda()
    m = tm.MeanSquaredError().cuda().set_dtype(torch.float64)
    m.update(p, t)
    ref = ((p.double() - t.double()) ** 2).mean()
    torch.testing.assert_close(m.compute(), ref, rtol=1e-6, atol=1e-9)
    # inputs that record autograd take the eager path (differentiable result)
    q = p.clone().requires_grad_(True)
    m2 = tm.MeanSquaredError().cuda()
    out = m2(q, t)
    out.backward()
    assert q.grad is not None
