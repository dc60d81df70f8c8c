"""gfx950 regression map-reduce kernel vs the fp32/fp64 PyTorch reference of the same sums, and GPU
functional/module results vs CPU."""
import pytest
import torch

from torchmetrics_forked_amd import ops
from torchmetrics_forked_amd.ops import regression as K

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_native(device):
    ops.require()


def _ref_table(p, t, op, param):
    cdt = torch.float64 if p.dtype == torch.float64 else torch.float32
    p, t = p.to(cdt), t.to(cdt)
    d = p - t
    chans = [p, t, p * p, t * t, p * t, d * d, d.abs(), K._eager_op(op, p, t, param)]
    return torch.stack([c.double().sum(0) for c in chans])


@pytest.mark.parametrize("op", range(8))
@pytest.mark.parametrize("shape", [(1,), (1000003, 1), (4097, 3), (2000, 64), (513, 100), (300, 1000)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64, torch.bfloat16, torch.float16])
def test_regression_sums(op, shape, dtype):
    g = torch.Generator().manual_seed(sum(shape) + op)
    p = (torch.rand(*shape, generator=g) + 0.1).to(dtype)
    t = (torch.rand(*shape, generator=g) + 0.1).to(dtype)
    param = 1.5 if op in (K.OP_MINKOWSKI, K.OP_TWEEDIE) else 0.0
    out = K.regression_sums(p.cuda(), t.cuda(), op, param).cpu()
    ref = _ref_table(p if p.ndim == 2 else p.unsqueeze(1), t if t.ndim == 2 else t.unsqueeze(1), op, param)
    assert out.shape == ref.shape
    rtol = 1e-9 if dtype == torch.float64 else 2e-5
    assert torch.allclose(out, ref, rtol=rtol, atol=1e-6), (out - ref).abs().max()


def test_regression_functional_gpu_vs_cpu():
    import torchmetrics_forked_amd.functional.regression as FR

    g = torch.Generator().manual_seed(0)
    p, t = torch.rand(10000, generator=g) + 0.1, torch.rand(10000, generator=g) + 0.1
    for fn in (FR.mean_squared_error, FR.mean_absolute_error, FR.mean_absolute_percentage_error,
               FR.symmetric_mean_absolute_percentage_error, FR.weighted_mean_absolute_percentage_error,
               FR.mean_squared_log_error, FR.log_cosh_error, FR.r2_score, FR.explained_variance, FR.pearson_corrcoef,
               FR.concordance_corrcoef, FR.relative_squared_error):
        a, b = fn(p.cuda(), t.cuda()).cpu(), fn(p, t)
        assert torch.allclose(a.double(), b.double(), rtol=1e-4, atol=1e-6), (fn.__name__, a, b)
    assert torch.allclose(FR.minkowski_distance(p.cuda(), t.cuda(), 3).cpu(), FR.minkowski_distance(p, t, 3), rtol=1e-4)
    assert torch.allclose(FR.tweedie_deviance_score(p.cuda(), t.cuda(), 1.5).cpu(), FR.tweedie_deviance_score(p, t, 1.5), rtol=1e-4)
    assert torch.allclose(FR.spearman_corrcoef(p.cuda(), t.cuda()).cpu(), FR.spearman_corrcoef(p, t), atol=1e-5)
    assert torch.allclose(FR.kendall_rank_corrcoef(p[:3000].cuda(), t[:3000].cuda()).cpu(),
                          FR.kendall_rank_corrcoef(p[:3000], t[:3000]), atol=1e-5)


def test_regression_modules_gpu():
    import torchmetrics_forked_amd.regression as RG

    g = torch.Generator().manual_seed(1)
    batches = [(torch.randn(4096, 3, generator=g), torch.randn(4096, 3, generator=g)) for _ in range(3)]
    for cls, kw in ((RG.MeanSquaredError, {"num_outputs": 3}), (RG.R2Score, {"num_outputs": 3}),
                    (RG.PearsonCorrCoef, {"num_outputs": 3}), (RG.ConcordanceCorrCoef, {"num_outputs": 3}),
                    (RG.LogCoshError, {"num_outputs": 3})):
        mg, mc = cls(**kw).cuda(), cls(**kw)
        for p, t in batches:
            mg.update(p.cuda(), t.cuda())
            mc.update(p, t)
        a, b = mg.compute().cpu(), mc.compute()
        assert torch.allclose(a.double(), b.double(), rtol=1e-4, atol=1e-6), (cls.__name__, a, b)


def test_pearson_inplace_update_gpu():
    """In-place native update (sums + merge kernel) vs the CPU module: 1-D and fp64 inputs, forward(), states."""
    import torchmetrics_forked_amd.regression as RG

    g = torch.Generator().manual_seed(7)
    for dtype in (torch.float32, torch.float64):
        mg, mc = RG.PearsonCorrCoef().cuda(), RG.PearsonCorrCoef()
        for i in range(4):
            p = (torch.randn(50000, generator=g) * 3 + 1).to(dtype)
            t = (0.5 * p + torch.randn(50000, generator=g, dtype=dtype)).to(dtype)
            bg = mg(p.cuda(), t.cuda())
            bc = mc(p, t)
            assert torch.allclose(bg.cpu().double(), bc.double(), rtol=1e-5, atol=1e-6)
        for name in ("mean_x", "mean_y", "var_x", "var_y", "corr_xy", "n_total"):
            a, b = getattr(mg, name).cpu().double(), getattr(mc, name).double()
            assert torch.allclose(a, b, rtol=1e-5, atol=1e-5), (name, a, b)
        assert torch.allclose(mg.compute().cpu().double(), mc.compute().double(), rtol=1e-5)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16, torch.float64])
@pytest.mark.parametrize("op", range(8))
def test_regression_sums_single_column(dtype, op):
    """D == 1 sums (aligned and offset views, odd N) vs an fp64 CPU reference; repeated calls are bitwise equal."""
    g = torch.Generator().manual_seed(op)
    N = 1_000_003
    p = (torch.rand(N + 1, generator=g) * 2 + 0.1).to(dtype)
    t = (torch.rand(N + 1, generator=g) * 2 + 0.1).to(dtype)
    param = 1.5 if op in (5, 7) else 0.0
    pg, tg = p.cuda(), t.cuda()
    flat = torch.ops.tmx.regression_sums(pg[:N].unsqueeze(1), tg[:N].unsqueeze(1), op, param)
    again = torch.ops.tmx.regression_sums(pg[:N].unsqueeze(1), tg[:N].unsqueeze(1), op, param)
    tiled = torch.ops.tmx.regression_sums(pg[1:].unsqueeze(1), tg[1:].unsqueeze(1), op, param)  # 2-B/4-B offset: tiled
    ref_tiled = torch.ops.tmx.regression_sums(pg[1 : N + 1].unsqueeze(1), tg[1 : N + 1].unsqueeze(1), op, param)
    assert torch.equal(flat, again)
    assert flat.shape == (8, 1)
    pc, tc = p[:N].double(), t[:N].double()
    d = pc - tc
    ref = torch.stack([pc.sum(), tc.sum(), (pc * pc).sum(), (tc * tc).sum(), (pc * tc).sum(), (d * d).sum(), d.abs().sum()])
    torch.testing.assert_close(flat[:7, 0].cpu(), ref, rtol=1e-4 if dtype != torch.float64 else 1e-10, atol=1e-6)
    assert tiled.shape == ref_tiled.shape == (8, 1)


@pytest.mark.parametrize("cls", ["MeanMetric", "SumMetric", "MaxMetric", "MinMetric"])
@pytest.mark.parametrize("strategy", ["warn", "ignore", "error", 0.5])
def test_aggregation_nan_policy_without_host_sync(cls, strategy):
    """GPU aggregation: NaN policy applied on device (neutralised entries, deferred warn / error at compute); the
    values match the CPU module, Python-scalar values and weights included."""
    import warnings

    import torchmetrics_forked_amd as tm

    mk = getattr(tm.aggregation, cls)
    mg, mc = mk(nan_strategy=strategy).cuda(), mk(nan_strategy=strategy)
    g = torch.Generator().manual_seed(2)
    batches = [torch.randn(100, generator=g), torch.randn(50, generator=g)]
    batches[1][[3, 17]] = float("nan")
    if strategy == "error":
        mg.update(batches[1].cuda())
        with pytest.raises(RuntimeError, match="nan"):
            mg.compute()
        return
    with warnings.catch_warnings(record=True) as wg:
        warnings.simplefilter("always")
        for b in batches:
            if cls == "MeanMetric":
                mg.update(b.cuda(), 2.0)
                mc.update(b, 2.0)
            else:
                mg.update(b.cuda())
                mc.update(b)
        mg.update(1.5)
        mc.update(1.5)
        out_g = mg.compute().cpu()
    torch.testing.assert_close(out_g, mc.compute(), rtol=1e-6, atol=1e-6)
    warned = any("nan" in str(w.message) for w in wg)
    assert warned == (strategy == "warn")
