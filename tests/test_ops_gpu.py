"""Numerics of the gfx950 HIP kernels vs the eager PyTorch (CPU) implementation of the same op.

Every op in ``torchmetrics_forked_amd.ops.classification`` is run on ``cuda:0`` (native library, mandatory) and
on CPU (eager reference path) with identical inputs; integer states must match exactly, float reductions to
fp64 rounding.
"""
import pytest
import torch

from torchmetrics_forked_amd import ops
from torchmetrics_forked_amd.ops import classification as K

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_native(device):
    ops.require()


def _both(fn, *tensors, **kw):
    """Run ``fn`` on (cuda copies, cpu copies); return the mutated/returned tensors of both."""
    gpu = [t.cuda() if isinstance(t, torch.Tensor) else t for t in tensors]
    cpu = [t.clone() if isinstance(t, torch.Tensor) else t for t in tensors]
    rg = fn(*gpu, **kw)
    rc = fn(*cpu, **kw)
    torch.cuda.synchronize()
    return gpu, cpu, rg, rc


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
def test_range_flag(dtype):
    x = torch.rand(10000).to(dtype)
    assert int(K.range_flag(x.cuda()).item()) == 0
    x[1234] = 1.5
    assert int(K.range_flag(x.cuda()).item()) == 1
    x[1234] = float("nan")
    assert int(K.range_flag(x.cuda()).item()) == 1


@pytest.mark.parametrize("minlength", [7, 1000, 70000])
def test_bincount(minlength):
    x = torch.randint(0, minlength, (200000,))
    out = torch.ops.tmx.bincount(x.cuda(), minlength)
    assert torch.equal(out.cpu(), torch.bincount(x, minlength=minlength))


@pytest.mark.parametrize("C", [5, 33, 1000])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16, torch.int64])
@pytest.mark.parametrize("ignore_index", [None, 2])
def test_mc_confmat(C, dtype, ignore_index):
    N = 5000
    preds = torch.randint(0, C, (N,)) if dtype == torch.int64 else torch.randn(N, C).to(dtype)
    target = torch.randint(0, C, (N,))
    if ignore_index is not None:
        target[::7] = ignore_index
    g, c, _, _ = _both(K.mc_confmat_update, preds, target, torch.zeros(C, C, dtype=torch.long), ignore_index)
    assert torch.equal(g[2].cpu(), c[2])


@pytest.mark.parametrize("L", [1, 6])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.int64])
@pytest.mark.parametrize("logits", [False, True])
def test_binary_stats(L, dtype, logits):
    N = 4000
    if dtype == torch.int64:
        preds = torch.randint(0, 2, (N, L, 3))
    else:
        preds = (torch.randn(N, L, 3) if logits else torch.rand(N, L, 3)).to(dtype)
    target = torch.randint(0, 2, (N, L, 3))
    target[::11] = -1
    g, c, _, _ = _both(K.binary_stats_update, preds, target, torch.zeros(L, 4, dtype=torch.long), L, 0.5, -1)
    assert torch.equal(g[2].cpu(), c[2])


@pytest.mark.parametrize("C", [4, 257, 1000])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("probs", [False, True])
def test_curve_hist_multiclass(C, dtype, probs):
    N = 3000
    x = torch.randn(N, C)
    preds = (x.softmax(1) if probs else x).to(dtype)
    target = torch.randint(0, C, (N,))
    target[::13] = -1
    hist = torch.zeros(C, 2, K.N_CODES, dtype=torch.long)
    cm = torch.zeros(C, C, dtype=torch.long)
    g, c, _, _ = _both(K.curve_hist_update, preds, target, hist, "multiclass", -1, cm)
    # softmax rounding of the fused fp32 kernel may flip a handful of bf16 roundings vs ATen's softmax
    diff = (g[2].cpu() - c[2]).abs().sum().item()
    assert diff <= max(8, int(1e-3 * N * C)), diff
    assert g[2].sum().item() == c[2].sum().item()
    assert torch.equal(g[5].cpu(), c[5])  # fused argmax confusion matrix is exact
    red_g = K.curve_hist_reduce(g[2]).cpu()
    red_c = K.curve_hist_reduce(g[2].cpu())
    torch.testing.assert_close(red_g, red_c, rtol=1e-12, atol=1e-12, equal_nan=True)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_curve_hist_multilabel(dtype):
    N, L = 2000, 7
    preds = torch.randn(N, L, 2).to(dtype)
    target = torch.randint(0, 2, (N, L, 2))
    target[::5, 0] = -1
    hist = torch.zeros(L, 2, K.N_CODES, dtype=torch.long)
    g, c, _, _ = _both(K.curve_hist_update, preds, target, hist, "multilabel", -1)
    assert torch.equal(g[2].cpu(), c[2])


@pytest.mark.parametrize("task,C", [("multiclass", 10), ("multilabel", 5), ("binary", 1)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_binned_curve(task, C, dtype):
    N, T = 3000, 11
    thr = torch.linspace(0, 1, T)
    if task == "multiclass":
        preds, target = torch.randn(N, C).softmax(1).to(dtype), torch.randint(0, C, (N,))
    else:
        preds, target = torch.rand(N, C, 1).to(dtype), torch.randint(0, 2, (N, C, 1))
    cm = torch.zeros(T, C, 2, 2, dtype=torch.long)
    g, c, _, _ = _both(K.binned_curve_update, preds, target, thr, cm, task, None)
    assert torch.equal(g[3].cpu(), c[3])


def test_module_auroc_confmat_gpu_matches_cpu():
    import torchmetrics_forked_amd as tm

    C, N = 100, 8192
    logits = torch.randn(N, C).bfloat16()
    target = torch.randint(0, C, (N,))
    out = []
    for dev in ("cuda", "cpu"):
        coll = tm.MetricCollection({"auroc": tm.MulticlassAUROC(num_classes=C), "cm": tm.MulticlassConfusionMatrix(num_classes=C)}).to(dev)
        for i in range(4):
            coll.update(logits[i::4].to(dev), target[i::4].to(dev))
        out.append({k: v.cpu() for k, v in coll.compute().items()})
    assert torch.equal(out[0]["cm"], out[1]["cm"])
    assert abs(out[0]["auroc"].item() - out[1]["auroc"].item()) < 1e-4


def _rare_rows(x, probs):
    """Sprinkle the rows the row pass hands to its rare-row kernel: NaN, +inf, all -inf, a single -inf, tied maxima."""
    N, C = x.shape
    x[5::97, 3] = float("nan")
    x[11::131, (C // 2)] = float("inf")
    x[17::211] = float("-inf")
    x[13::89, 1] = float("-inf")
    x[23::53, 0] = x[23::53, 2] = 0.75 if probs else 9.0
    return x


@pytest.mark.parametrize("C", [10, 64, 100, 512, 520, 1000, 1001])
@pytest.mark.parametrize("probs", [False, True])
def test_curve_hist_multiclass_rare_rows(C, probs):
    """Rows with NaN / inf take mc_slow_rows_kernel: torch semantics (all-NaN softmax, first-NaN arg-max)."""
    N = 4000
    x = torch.randn(N, C)
    x = _rare_rows(x.softmax(1) if probs else x, probs).bfloat16()
    target = torch.randint(0, C, (N,))
    target[::19] = -1
    hist = torch.zeros(C, 2, K.N_CODES, dtype=torch.long)
    cm = torch.zeros(C, C, dtype=torch.long)
    g, c, _, _ = _both(K.curve_hist_update, x, target, hist, "multiclass", -1, cm)
    assert torch.equal(g[5].cpu(), c[5])  # confusion matrix incl. NaN / all -inf rows is exact
    diff = (g[2].cpu() - c[2]).abs().sum().item()
    assert diff <= max(8, int(1e-3 * N * C)), diff
    assert g[2].sum().item() == c[2].sum().item()


def test_curve_speculation_flips_across_batches():
    """The persistent mode word speculates softmax-vs-raw from the previous batch; a wrong guess is redone (FIXUP)."""
    import torchmetrics_forked_amd as tm

    C, N = 520, 3000
    gen = torch.Generator().manual_seed(3)
    batches = []
    for kind in ("logits", "probs", "probs", "logits", "probs_nan", "logits", "small_logits"):
        x = torch.randn(N, C, generator=gen)
        if kind == "probs":
            x = x.softmax(1)
        elif kind == "probs_nan":
            x = x.softmax(1)
            x[7, 3] = float("nan")  # one NaN makes the reference softmax the whole batch
        elif kind == "small_logits":
            x = x.abs().clamp(max=1.0) * torch.where(torch.rand(N, C, generator=gen) < 0.5, -1.0, 1.0)  # max <= 1, some < 0
        batches.append((x.bfloat16(), torch.randint(0, C, (N,), generator=gen)))
    res = []
    for dev in ("cuda", "cpu"):
        m = tm.MulticlassAUROC(num_classes=C, average="macro").to(dev)
        cmm = tm.MulticlassConfusionMatrix(num_classes=C).to(dev)
        vals = []
        for x, t in batches:
            m.update(x.to(dev), t.to(dev))
            cmm.update(x.to(dev), t.to(dev))
            vals.append(m.compute().item())
        res.append((vals, cmm.compute().cpu()))
    assert torch.equal(res[0][1], res[1][1])
    for a, b in zip(res[0][0], res[1][0]):
        assert abs(a - b) < 1e-4, (res[0][0], res[1][0])


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("probs", [False, True])
@pytest.mark.parametrize("offset", [0, 1])
def test_curve_hist_binary(dtype, probs, offset):
    """Single-label path (LDS-privatised binary_hist_kernel; offset 1 = misaligned view -> element-wise kernel)."""
    N = 200_003
    x = torch.rand(N + offset) if probs else torch.randn(N + offset) * 3
    x[17::1001] = float("nan")
    preds = x.to(dtype)[offset:]
    target = torch.randint(0, 2, (N + offset,))[offset:]
    target[5::13] = -1
    hist = torch.zeros(1, 2, K.N_CODES, dtype=torch.long)
    g, c, _, _ = _both(K.curve_hist_update, preds.reshape(-1, 1, 1), target.reshape(-1, 1, 1), hist, "binary", -1)
    assert torch.equal(g[2].cpu(), c[2])


@pytest.mark.parametrize("L", [8, 64, 520, 1000])
@pytest.mark.parametrize("probs", [False, True])
def test_curve_hist_multilabel_two_pass(L, probs):
    """[N, L] multilabel scores take the two-pass route (ml_codes_kernel + class pass): per-element sigmoid,
    per-element targets with ignore_index, NaN scores skipped."""
    N = 3000
    x = torch.rand(N, L) if probs else torch.randn(N, L) * 2
    x[7::101, 3] = float("nan")
    preds = x.bfloat16()
    target = torch.randint(0, 2, (N, L))
    target[::11, :5] = -1
    hist = torch.zeros(L, 2, K.N_CODES, dtype=torch.long)
    g, c, _, _ = _both(K.curve_hist_update, preds, target, hist, "multilabel", -1)
    diff = (g[2].cpu() - c[2]).abs().sum().item()
    assert diff <= max(8, int(1e-4 * N * L)), diff  # CPU vs GPU expf may flip a rare bf16 rounding of the sigmoid
    assert g[2].sum().item() == c[2].sum().item()
    assert torch.equal(g[2][:, 1].sum(-1).cpu(), c[2][:, 1].sum(-1))  # positives per label exact


@pytest.mark.parametrize("task,C", [("binary", 1), ("multilabel", 5), ("multilabel", 300)])
def test_binned_curve_lds(task, C):
    """Element-wise binned histogram with LDS-privatised per-wave / per-block copies vs the CPU path."""
    N, T = 20_001, 101
    thr = torch.linspace(0, 1, T)
    preds = torch.rand(N, C, 1)
    target = torch.randint(0, 2, (N, C, 1))
    target[::9] = -1
    cm = torch.zeros(T, C, 2, 2, dtype=torch.long)
    g, c, _, _ = _both(K.binned_curve_update, preds, target, thr, cm, task, -1)
    assert torch.equal(g[3].cpu(), c[3])


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("probs", [False, True])
def test_multiclass_calibration_fused(dtype, probs):
    """Fused top-label calibration kernel (rounded softmax max, first arg-max, NaN rows) vs the CPU eager path."""
    import torchmetrics_forked_amd as tm

    N, C = 5000, 37
    x = torch.randn(N, C)
    x = x.softmax(1) if probs else x * 3
    x[11::97, 5] = float("nan")
    x[3::101, 1] = x[3::101].max(1).values  # exact ties at the maximum
    preds = x.to(dtype)
    target = torch.randint(0, C, (N,))
    target[::13] = -1
    out = []
    for dev in ("cuda", "cpu"):
        m = tm.MulticlassCalibrationError(num_classes=C, n_bins=15, norm="l1", ignore_index=-1).to(dev)
        m.update(preds.to(dev), target.to(dev))
        out.append((m.bins.cpu(), m.compute().cpu()))
    torch.testing.assert_close(out[0][0], out[1][0], rtol=1e-9, atol=1e-6, equal_nan=True)
    torch.testing.assert_close(out[0][1], out[1][1], rtol=1e-5, atol=1e-6, equal_nan=True)


def test_binary_calibration_bins():
    import torchmetrics_forked_amd as tm

    N = 100_003
    preds, target = torch.rand(N), torch.randint(0, 2, (N,))
    out = []
    for dev in ("cuda", "cpu"):
        m = tm.BinaryCalibrationError(n_bins=10, norm="l2").to(dev)
        m.update(preds.to(dev), target.to(dev))
        out.append((m.bins.cpu(), m.compute().cpu()))
    torch.testing.assert_close(out[0][0], out[1][0], rtol=1e-9, atol=1e-6)
    torch.testing.assert_close(out[0][1], out[1][1], rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("C,dtype", [(64, torch.float32), (512, torch.float32), (40, torch.bfloat16), (1000, torch.bfloat16),
                                     (1024, torch.float16), (96, torch.float64)])
def test_mc_confmat_vectorised(C, dtype):
    """Vectorised arg-max confusion matrix (4 rows in flight per wave): ties -> first index, NaN -> first NaN."""
    N = 9001
    x = torch.randn(N, C)
    x[3::17, 2] = x[3::17].max(1).values + 1
    x[3::17, 7] = x[3::17, 2]  # tie: class 2 must win
    x[5::29, C // 2] = float("nan")
    x[5::58, 1] = float("nan")  # two NaNs: the first wins
    target = torch.randint(0, C, (N,))
    target[::11] = 3
    g, c, _, _ = _both(K.mc_confmat_update, x.to(dtype), target, torch.zeros(C, C, dtype=torch.long), 3)
    assert torch.equal(g[2].cpu(), c[2])
