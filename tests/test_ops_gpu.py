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
    torch.manual_seed(1000 * C + (dtype == torch.float16) * 10 + int(probs))  # the moved-code count is data dependent
    x = torch.randn(N, C)
    preds = (x.softmax(1) if probs else x).to(dtype)
    target = torch.randint(0, C, (N,))
    target[::13] = -1
    hist = torch.zeros(C, 2, K.N_CODES, dtype=torch.long)
    cm = torch.zeros(C, C, dtype=torch.long)
    g, c, _, _ = _both(K.curve_hist_update, preds, target, hist, "multiclass", -1, cm)
    # probabilities are coded from their raw bits: exact.  Logits: the fused softmax sums exp(x - max) in another fp32
    # order than ATen's, so a few elements land one 16-bit code away (pinned per element at <= 2e-5 / 1.5e-4 of the
    # elements by test_curve_hist_codes_vs_aten_softmax_same_device); each moved element changes two bins
    diff = (g[2].cpu() - c[2]).abs().sum().item()
    rate = 4e-5 if dtype == torch.bfloat16 else 3e-4  # 2x the pinned per-element rate: headroom for unseeded data
    assert diff == 0 if probs else diff <= max(8, int(2 * rate * N * C)), diff
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
    # ~4 of the 819200 bf16 softmax scores may sit one code away from ATen's (see above); each moves a class AUROC by
    # at most (crossed pairs) / (P N) ~ 1.5e-6, the macro mean by ~1e-8
    assert abs(out[0]["auroc"].item() - out[1]["auroc"].item()) < 1e-6


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
    # the sprinkled NaN / inf make even the probability batches softmax batches (reference rule): the logits bound
    assert diff <= max(8, int(2 * 4e-5 * N * C)), diff  # see test_curve_hist_multiclass (2x headroom: unseeded data)
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
        assert abs(a - b) < 2e-5, (res[0][0], res[1][0])


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
    x = torch.randn(N, C, generator=torch.Generator().manual_seed(11))
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
    if dtype == torch.float32 or probs:
        torch.testing.assert_close(out[0][0], out[1][0], rtol=1e-9, atol=1e-6, equal_nan=True)
        torch.testing.assert_close(out[0][1], out[1][1], rtol=1e-5, atol=1e-6, equal_nan=True)
    else:
        # 16-bit logits: the softmax sum is reduced in a different order than ATen's, so a rounded confidence can
        # land on the other side of a bin edge now and then (parity: a handful of samples, same metric value)
        assert (out[0][0][0] - out[1][0][0]).abs().sum().item() <= 6
        torch.testing.assert_close(out[0][1], out[1][1], rtol=0, atol=2e-3, equal_nan=True)


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
                                     (1024, torch.float16), (96, torch.float64), (10, torch.bfloat16), (17, torch.float32),
                                     (100, torch.bfloat16), (128, torch.float64), (33, torch.float16), (3, torch.float32)])
def test_mc_confmat_vectorised(C, dtype):
    """Vectorised arg-max confusion matrix (4 rows in flight per wave): ties -> first index, NaN -> first NaN."""
    N = 9001
    x = torch.randn(N, C)
    a, b = (2, 7) if C > 7 else (0, C - 1)
    x[3::17, a] = x[3::17].max(1).values + 1
    x[3::17, b] = x[3::17, a]  # tie: class a must win
    x[5::29, C // 2] = float("nan")
    x[5::58, 1] = float("nan")  # two NaNs: the first wins
    target = torch.randint(0, C, (N,))
    target[::11] = 3
    g, c, _, _ = _both(K.mc_confmat_update, x.to(dtype), target, torch.zeros(C, C, dtype=torch.long), 3)
    assert torch.equal(g[2].cpu(), c[2])


def _stat_oracle(preds, target, C, ignore_index, micro):
    cm = torch.zeros(C, C, dtype=torch.long)
    K.mc_confmat_update(preds.cpu(), target.cpu(), cm, ignore_index)
    tp = cm.diag()
    fp, fn = cm.sum(0) - tp, cm.sum(1) - tp
    tn = cm.sum() - (tp + fp + fn)
    out = [tp, fp, tn, fn]
    return [o.sum().reshape(1) for o in out] if micro else out


@pytest.mark.parametrize(
    ("C", "dtype"),
    [(3, torch.float32), (10, torch.bfloat16), (40, torch.bfloat16), (64, torch.float16), (100, torch.float32),
     (1000, torch.bfloat16), (1001, torch.bfloat16), (1024, torch.float64), (6000, torch.float32)],
)
@pytest.mark.parametrize("micro", [False, True])
@pytest.mark.parametrize("ignore_index", [None, 1, -100])
def test_mc_stat_scores_fused(C, dtype, micro, ignore_index):
    """Fused arg-max -> tp/fp/tn/fn into the states (LDS-privatised, global-atomic and micro tiers; ticket word
    returns to zero so consecutive updates accumulate)."""
    torch.manual_seed(C)
    size = 1 if micro else C
    states = [torch.zeros(size, dtype=torch.long, device="cuda") for _ in range(4)]
    ticket = torch.zeros(K.GRID_SLOTS, dtype=torch.long, device="cuda")
    expect = [torch.zeros(size, dtype=torch.long) for _ in range(4)]
    for N in (1, 777, 20000):
        x = torch.randn(N, C).to(dtype)
        t = torch.randint(0, C, (N,))
        if ignore_index is not None:
            t[::7] = ignore_index
        K.mc_stat_scores_update(x.cuda(), t.cuda(), C, *states, ticket, ignore_index, micro)
        for e, o in zip(expect, _stat_oracle(x, t, C, ignore_index, micro)):
            e += o
        torch.cuda.synchronize()
        assert int(ticket.abs().sum().item()) == 0
        for s, e in zip(states, expect):
            assert torch.equal(s.cpu(), e)


@pytest.mark.parametrize("C", [5, 300])
def test_mc_stat_scores_labels_and_flags(C):
    """Integer predictions, and the deferred range flags (bad target / bad pred) raised at compute."""
    N = 5000
    p = torch.randint(0, C, (N,))
    t = torch.randint(0, C, (N,))
    states = [torch.zeros(C, dtype=torch.long, device="cuda") for _ in range(4)]
    ticket = torch.zeros(K.GRID_SLOTS, dtype=torch.long, device="cuda")
    et = torch.zeros(1, dtype=torch.int32, device="cuda")
    ep = torch.zeros(1, dtype=torch.int32, device="cuda")
    K.mc_stat_scores_update(p.cuda(), t.cuda(), C, *states, ticket, None, False, et, ep)
    for s, e in zip(states, _stat_oracle(p, t, C, None, False)):
        assert torch.equal(s.cpu(), e)
    assert int(et.item()) == 0 and int(ep.item()) == 0
    t[17] = C
    p[33] = -1
    K.mc_stat_scores_update(p.cuda(), t.cuda(), C, *states, ticket, None, False, et, ep)
    assert int(et.item()) == 1 and int(ep.item()) == 1


def test_multiclass_modules_fused_path():
    """Accuracy / F1 / ConfusionMatrix modules on the fused path agree with the CPU path over several updates, and
    an out-of-range target raises at compute (deferred validation)."""
    from torchmetrics_forked_amd.classification import MulticlassAccuracy, MulticlassConfusionMatrix, MulticlassF1Score

    C = 37
    for cls, kw in ((MulticlassAccuracy, {"average": "macro"}), (MulticlassAccuracy, {"average": "micro"}),
                    (MulticlassF1Score, {"average": "weighted", "ignore_index": 2}), (MulticlassConfusionMatrix, {})):
        mg, mc = cls(num_classes=C, **kw).cuda(), cls(num_classes=C, **kw)
        for _ in range(3):
            x = torch.randn(4000, C)
            t = torch.randint(0, C, (4000,))
            mg.update(x.cuda(), t.cuda())
            mc.update(x, t)
        torch.testing.assert_close(mg.compute().cpu(), mc.compute())
        bad = cls(num_classes=C, **kw).cuda()
        t = torch.randint(0, C, (100,))
        t[5] = C + 3
        bad.update(torch.randn(100, C).cuda(), t.cuda())
        with pytest.raises(RuntimeError, match="unique values in `target`"):
            bad.compute()


def _bin_case(shape, dtype, logits, ignore_index, seed):
    g = torch.Generator().manual_seed(seed)
    if dtype == torch.int64:
        p = torch.randint(0, 2, shape, generator=g)
    else:
        p = (torch.randn(shape, generator=g) * 3 if logits else torch.rand(shape, generator=g)).to(dtype)
    t = torch.randint(0, 2, shape, generator=g)
    if ignore_index is not None:
        t.view(-1)[::5] = ignore_index
    return p, t


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16, torch.float64, torch.int64])
@pytest.mark.parametrize(
    ("shape", "L"),
    [((1,), 1), ((7,), 1), ((1001,), 1), ((1 << 20) + 3, 1),
     ((333, 3), 3), ((4096, 8), 8), ((2048, 1000), 1000), ((100, 5, 4), 5), ((64, 6, 16), 6), ((50, 3000), 3000)],
)
@pytest.mark.parametrize("logits", [False, True])
@pytest.mark.parametrize("ignore_index", [None, -1])
def test_binary_stats_fused(dtype, shape, L, logits, ignore_index):
    """One-launch binary / multilabel stats (raw and sigmoid counts, last workgroup picks) vs the eager path, over
    three updates so the scratch / ticket reset is exercised."""
    if isinstance(shape, int):
        shape = (shape,)
    states = tuple(torch.zeros(L, dtype=torch.long, device="cuda") for _ in range(4))
    scratch = torch.zeros(6 * L + K.GRID_SLOTS, dtype=torch.long, device="cuda")
    expect = torch.zeros(L, 4, dtype=torch.long)
    for seed in range(3):
        p, t = _bin_case(shape, dtype, logits and seed != 1, ignore_index, seed)
        K.binary_stats_fused(p.cuda(), t.cuda(), states, scratch, L, 0.3, ignore_index)
        K.binary_stats_update(p, t, expect, L, 0.3, ignore_index)
        torch.cuda.synchronize()
        assert int(scratch.abs().sum().item()) == 0
        got = torch.stack([s.cpu() for s in states], dim=1)
        assert torch.equal(got, expect), (got - expect).abs().max()


def test_binary_stats_fused_misaligned_and_flags():
    L = 8
    p = torch.rand(4097, L)
    t = torch.randint(0, 2, (4097, L))
    pg, tg = p.cuda()[1:], t.cuda()[1:]  # 32-B offset rows: still 16-B aligned; then a 4-B offset view
    states = tuple(torch.zeros(L, dtype=torch.long, device="cuda") for _ in range(4))
    scratch = torch.zeros(6 * L + K.GRID_SLOTS, dtype=torch.long, device="cuda")
    K.binary_stats_fused(pg, tg, states, scratch, L, 0.5, None)
    expect = torch.zeros(L, 4, dtype=torch.long)
    K.binary_stats_update(p[1:], t[1:], expect, L, 0.5, None)
    flat_p, flat_t = p.reshape(-1)[1:4097 * L - 7], t.reshape(-1)[1:4097 * L - 7]
    s1 = tuple(torch.zeros(1, dtype=torch.long, device="cuda") for _ in range(4))
    sc1 = torch.zeros(6 + K.GRID_SLOTS, dtype=torch.long, device="cuda")
    K.binary_stats_fused(flat_p.cuda(), flat_t.cuda(), s1, sc1, 1, 0.5, None)
    e1 = torch.zeros(1, 4, dtype=torch.long)
    K.binary_stats_update(flat_p, flat_t, e1, 1, 0.5, None)
    torch.cuda.synchronize()
    assert torch.equal(torch.stack([s.cpu() for s in states], 1), expect)
    assert torch.equal(torch.stack([s.cpu() for s in s1], 1), e1)
    et = torch.zeros(1, dtype=torch.int32, device="cuda")
    ep = torch.zeros(1, dtype=torch.int32, device="cuda")
    lp = torch.randint(0, 2, (1000,))
    lt = torch.randint(0, 2, (1000,))
    K.binary_stats_fused(lp.cuda(), lt.cuda(), s1, sc1, 1, 0.5, -1, et, ep)
    assert int(et.item()) == 0 and int(ep.item()) == 0
    lt[10] = -1  # ignored: fine
    K.binary_stats_fused(lp.cuda(), lt.cuda(), s1, sc1, 1, 0.5, -1, et, ep)
    assert int(et.item()) == 0
    lt[11] = 2
    lp[12] = 3
    K.binary_stats_fused(lp.cuda(), lt.cuda(), s1, sc1, 1, 0.5, -1, et, ep)
    assert int(et.item()) == 1 and int(ep.item()) == 1


def test_binary_multilabel_modules_fused_path():
    from torchmetrics_forked_amd.classification import BinaryAccuracy, BinaryF1Score, MultilabelF1Score, MultilabelPrecision

    for mk, shape in ((lambda: BinaryAccuracy(), (5000,)), (lambda: BinaryF1Score(ignore_index=-1), (5000,)),
                      (lambda: MultilabelF1Score(num_labels=12), (3000, 12)),
                      (lambda: MultilabelPrecision(num_labels=12, average="micro"), (3000, 12))):
        mg, mc = mk().cuda(), mk()
        for seed in range(3):
            p, t = _bin_case(shape, torch.float32, seed == 2, None, seed)
            mg.update(p.cuda(), t.cuda())
            mc.update(p, t)
        torch.testing.assert_close(mg.compute().cpu(), mc.compute())
        bad = mk().cuda()
        p, t = _bin_case(shape, torch.float32, False, None, 0)
        t.view(-1)[3] = 7
        bad.update(p.cuda(), t.cuda())
        with pytest.raises(RuntimeError, match="`target`"):
            bad.compute()


@pytest.mark.parametrize(
    "kind", ["binary_hist", "binary_hist_lds", "binary_binned", "multilabel_hist", "multilabel_binned", "multiclass_binned"]
)
def test_curve_value_checks_in_kernel(kind):
    """Curve metrics fold the target value check into the histogram pass (device flag, raised at compute) and write
    binned counts straight into the state; results match the CPU module."""
    from torchmetrics_forked_amd.classification import BinaryAUROC, MulticlassAUROC, MultilabelAUROC

    g = torch.Generator().manual_seed(5)
    if kind.startswith("binary"):
        mk = lambda: BinaryAUROC(thresholds=50 if "binned" in kind else None)  # noqa: E731
        n = 40000 if kind == "binary_hist_lds" else 3001
        p = torch.rand(n, generator=g)
        p = p.bfloat16() if "hist" in kind else p
        t = torch.randint(0, 2, (n,), generator=g)
        bad_t = t.clone()
        bad_t[7] = 2
    elif kind.startswith("multilabel"):
        L = 16 if kind == "multilabel_hist" else 5
        mk = lambda: MultilabelAUROC(num_labels=L, thresholds=50 if "binned" in kind else None)  # noqa: E731
        p = torch.rand(2000, L, generator=g)
        p = p.bfloat16() if "hist" in kind else p
        t = torch.randint(0, 2, (2000, L), generator=g)
        bad_t = t.clone()
        bad_t[3, 1] = -4
    else:
        C = 7
        mk = lambda: MulticlassAUROC(num_classes=C, thresholds=50)  # noqa: E731
        p = torch.randn(3000, C, generator=g).softmax(1)
        t = torch.randint(0, C, (3000,), generator=g)
        bad_t = t.clone()
        bad_t[11] = C
    mg, mc = mk().cuda(), mk()
    for _ in range(2):
        mg.update(p.cuda(), t.cuda())
        mc.update(p, t)
    torch.testing.assert_close(mg.compute().cpu().float(), mc.compute().float(), atol=1e-4, rtol=1e-4)
    bad = mk().cuda()
    bad.update(p.cuda(), bad_t.cuda())
    with pytest.raises(RuntimeError):
        bad.compute()


@pytest.mark.parametrize("C,dtype", [(40, torch.float32), (40, torch.bfloat16), (1000, torch.bfloat16), (512, torch.float16),
                                     (1024, torch.float32)])
@pytest.mark.parametrize("probs", [False, True])
def test_multiclass_calibration_one_pass(C, dtype, probs):
    """One-pass fused calibration (raw rows, in-kernel ignore filtering and softmax decision, both modes binned) vs
    the CPU module over several batches, plus the deferred target range check."""
    import torchmetrics_forked_amd as tm

    g = torch.Generator().manual_seed(C)
    mg = tm.MulticlassCalibrationError(num_classes=C, n_bins=15, ignore_index=-1).cuda()
    mc = tm.MulticlassCalibrationError(num_classes=C, n_bins=15, ignore_index=-1)
    for b in range(3):
        x = torch.randn(3001, C, generator=g)
        x = x.softmax(1) if probs else x * 3
        if b == 1:
            x[3::101, 1] = x[3::101].max(1).values  # exact ties at the maximum
            if not probs:
                x[11::97, 5] = float("nan")
        preds = x.to(dtype)
        target = torch.randint(0, C, (3001,), generator=g)
        target[::13] = -1
        mg.update(preds.cuda(), target.cuda())
        mc.update(preds, target)
    bg, bc = mg.bins.cpu(), mc.bins
    if dtype == torch.float32 or probs:
        torch.testing.assert_close(bg[0], bc[0], rtol=0, atol=0)
        # fp32 logits: 1 / sum(exp) differs from ATen's softmax in the last bit (other summation order)
        torch.testing.assert_close(bg, bc, rtol=1e-6, atol=1e-6, equal_nan=True)
    else:
        assert (bg[0] - bc[0]).abs().sum().item() <= 8
    torch.testing.assert_close(mg.compute().cpu(), mc.compute(), rtol=0, atol=2e-3, equal_nan=True)
    if C > 128 * (16 // preds.element_size()):
        return  # unfused fallback: the eager check counts unique targets (reference semantics), no range flag
    bad = tm.MulticlassCalibrationError(num_classes=C).cuda()
    t = torch.randint(0, C, (64,))
    t[9] = C
    bad.update(torch.randn(64, C).to(dtype).cuda(), t.cuda())
    with pytest.raises(RuntimeError):
        bad.compute()


@pytest.mark.parametrize("kind", ["linspace", "irregular", "single"])
def test_binned_bucket_guess_exact(kind):
    """Bucket lookup (arithmetic guess + neighbour check + binary-search fallback) matches the eager path, with
    scores exactly on thresholds, outside [0, 1] neighbours, and NaN."""
    T = {"linspace": 101, "irregular": 37, "single": 1}[kind]
    if kind == "irregular":
        thr = torch.sort(torch.rand(T, generator=torch.Generator().manual_seed(1)) ** 3).values
    else:
        thr = torch.linspace(0, 1, T)
    p = torch.rand(20000, generator=torch.Generator().manual_seed(2))
    p[:T] = thr  # exactly on each threshold
    p[T : T + 3] = torch.tensor([0.0, 1.0, 0.5])
    t = torch.randint(0, 2, (20000,), generator=torch.Generator().manual_seed(3))
    for tensor_in in (p, p.reshape(4000, 5)):
        C = 1 if tensor_in.ndim == 1 else 5
        tt = t.reshape(tensor_in.shape)
        cm = torch.zeros(T, C, 2, 2, dtype=torch.long)
        pin = tensor_in.reshape(-1, 1, 1) if C == 1 else tensor_in
        tin = tt.reshape(-1, 1, 1) if C == 1 else tt
        g, c, _, _ = _both(K.binned_curve_update, pin, tin, thr, cm, "binary" if C == 1 else "multilabel", None)
        assert torch.equal(g[3].cpu(), c[3])


@pytest.mark.parametrize("C", [3, 1000])
@pytest.mark.parametrize("span", ["narrow", "wide", "full", "empty"])
def test_curve_hist_reduce_tracked_range(C, span):
    """The range-limited reduction (chunks of 4096 codes from the top of the tracked range) equals the full-range
    reduction of the same histogram, for ranges inside one chunk, across chunks, the full range and an empty one."""
    g = torch.Generator().manual_seed(C)
    hist = torch.zeros(C, 2, K.N_CODES, dtype=torch.long)
    lo, hi = {"narrow": (16001, 16200), "wide": (3, 12345), "full": (0, K.N_CODES - 1), "empty": (K.N_CODES, -1)}[span]
    if hi >= lo:
        hist[:, :, lo : hi + 1] = torch.randint(0, 4, (C, 2, hi - lo + 1), generator=g) * (torch.rand(C, 2, hi - lo + 1, generator=g) < 0.3)
        hist[0, 1] = 0  # a class without positives (AP NaN, degenerate flag)
    rng = torch.tensor([lo, hi], dtype=torch.int32, device="cuda").repeat(C, 1)
    got = K.curve_hist_reduce(hist.cuda(), rng).cpu()
    full = K.curve_hist_reduce(hist.cuda()).cpu()
    ref = K.curve_hist_reduce(hist)
    torch.testing.assert_close(got, ref, rtol=1e-12, atol=1e-12, equal_nan=True)
    torch.testing.assert_close(full, ref, rtol=1e-12, atol=1e-12, equal_nan=True)
    summ = K.curve_summary(got.cuda()).cpu()
    torch.testing.assert_close(summ[:8], K.curve_summary(ref), rtol=1e-12, atol=1e-12, equal_nan=True)


def test_tracked_code_range_module():
    """The class pass widens the module's tracked code range to exactly the occupied codes; the range-limited compute
    equals the compute over a histogram of unknown range (recomputed) and the CPU path."""
    import torchmetrics_forked_amd as tm

    C = 100
    m = tm.MulticlassAUROC(num_classes=C, average=None).cuda()
    x = torch.randn(4096, C).bfloat16()
    t = torch.randint(0, C, (4096,))
    m.update(x.cuda(), t.cuda())
    rng = m._tracked_range().cpu()
    for c in (0, 17, C - 1):
        occ = (m.score_hist[c].amax(0) > 0).nonzero().flatten().cpu()
        assert rng[c].tolist() == [int(occ.min()), int(occ.max())]
    a = m.compute().cpu()
    m._invalidate_range()
    m._computed = None
    b = m.compute().cpu()
    cpu = tm.MulticlassAUROC(num_classes=C, average=None)
    cpu.update(x, t)
    torch.testing.assert_close(a, b, rtol=0, atol=0)
    torch.testing.assert_close(a, cpu.compute(), rtol=0, atol=2e-4)


def _hist_from_scores(scores, target, C):
    """Exact (class, label, 16-bit code) histogram of 16-bit scores in [0, 1] (-0.0 -> code 0)."""
    codes = scores.view(torch.int16).long() & 0x7FFF
    codes = torch.where(codes > 0x3FFF, torch.zeros_like(codes), codes)
    lab = (torch.arange(C, device=scores.device)[None, :] == target[:, None]).long()
    flat = (torch.arange(C, device=scores.device)[None, :] * 2 + lab) * K.N_CODES + codes
    h = torch.zeros(C, 2, K.N_CODES, dtype=torch.long, device=scores.device)
    h.view(-1).index_add_(0, flat.reshape(-1), torch.ones_like(flat.reshape(-1)))
    return h


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_curve_hist_codes_vs_aten_softmax_same_device(dtype):
    """Pinned bound of the fused softmax codes against ATen's GPU softmax of the same logits (what the reference
    computes).  The row pass sums exp(x - max) in a different fp32 order than ATen's warp softmax (64 lanes x 16
    sequential, xor butterfly 32..1; ``tools/probes/softmax_order_probe.py``), so a quotient within an ulp of a 16-bit
    rounding boundary can round to the neighbouring code.  Checked per element (the row pass's class-major codes):
    every difference is exactly one code, at most 2e-5 (bf16) / 1.5e-4 (fp16) of the elements differ (measured
    ~5e-6 / ~8e-5), and AUROC / AP over all classes equal the sort-based computation on ATen's scores to 1e-7."""
    from torchmetrics_forked_amd.functional.classification import _curve_engine as eng

    N, C = 65536, 1000
    g = torch.Generator(device="cuda").manual_seed(11)
    x = torch.randn(N, C, device="cuda", generator=g).to(dtype)
    t = torch.randint(0, C, (N,), device="cuda", generator=g)
    mode = torch.ones(2, dtype=torch.int32, device="cuda")  # speculate softmax (logits batch): no FIXUP pass
    state = torch.zeros(6, dtype=torch.int32, device="cuda")
    n_pad = (N + 31) // 32 * 32
    codes = torch.empty(C * n_pad, dtype=torch.int16, device="cuda")
    rows = torch.empty(2 * N, dtype=torch.int32, device="cuda")
    torch.ops.tmx.curve_mc_rowpass(x, t, mode, state, codes, rows, -1, False, None, None)
    kc = (codes.view(C, n_pad)[:, :N].t().int() & 0x3FFF)
    ref = torch.softmax(x, dim=1)
    rc = ref.view(torch.int16).int() & 0x7FFF
    diff = (kc - rc).abs()
    assert int(diff.max()) <= 1, int(diff.max())
    moved = int((diff != 0).sum())
    assert moved <= (2e-5 if dtype == torch.bfloat16 else 1.5e-4) * N * C, moved
    # the histogram built from these codes by the class pass, reduced, vs sorting ATen's scores
    hist = torch.zeros(C, 2, K.N_CODES, dtype=torch.long, device="cuda")
    K.curve_hist_update(x, t, hist, "multiclass", None)
    assert torch.equal(hist, _hist_from_scores(kc.to(torch.int16).view(dtype), t, C))
    red = K.curve_hist_reduce(hist)
    labels = torch.nn.functional.one_hot(t, C).bool()
    auc_s, ap_s, _, _ = eng.samples_scores(ref, labels)
    assert abs(red[:, 0].mean().item() - auc_s.mean().item()) <= 1e-7
    assert abs(red[:, 1].mean().item() - ap_s.mean().item()) <= 1e-7
    # classes without a moved score: the histogram reduction IS the sort-based result
    same = (diff.sum(0) == 0)
    torch.testing.assert_close(red[same, 0], auc_s[same], rtol=0, atol=1e-12)
    torch.testing.assert_close(red[same, 1], ap_s[same], rtol=0, atol=1e-12)


def _flip_batches(C, N, seed=5):
    gen = torch.Generator().manual_seed(seed)
    out = []
    for kind in ("logits", "probs", "probs", "logits", "nan_rows", "logits", "probs_nan", "logits"):
        x = torch.randn(N, C, generator=gen)
        if kind.startswith("probs"):
            x = x.softmax(1)
        if kind.endswith("nan") or kind == "nan_rows":
            x = _rare_rows(x, kind.startswith("probs"))
        out.append((x.bfloat16(), torch.randint(0, C, (N,), generator=gen)))
    return out


@pytest.mark.parametrize("strategy", ["warn", "ignore", "error"])
def test_cat_metric_gpu_defers_nan_drop(strategy):
    """CatMetric on the GPU: no host sync per update (NaN policy as a device flag, NaN entries dropped once by the
    first state consumer), same result as the CPU metric, including across forward() and state_dict()."""
    import warnings

    import torchmetrics_forked_amd as tm

    xs = [torch.tensor([1.0, float("nan"), 3.0]), torch.tensor([4.0]), torch.tensor([float("nan"), 6.0])]
    mg, mc = tm.aggregation.CatMetric(nan_strategy=strategy).cuda(), tm.aggregation.CatMetric(nan_strategy=strategy)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        if strategy == "error":
            mg.update(xs[0].cuda())
            with pytest.raises(RuntimeError, match="nan"):
                mg.compute()
            return
        mg.update(xs[0].cuda())
        out_fwd = mg(xs[1].cuda())
        mg.update(xs[2].cuda())
        mc.update(xs[0])
        ref_fwd = mc(xs[1])
        mc.update(xs[2])
        assert torch.equal(out_fwd.cpu(), ref_fwd)
        assert torch.equal(mg.compute().cpu(), mc.compute())


@pytest.mark.parametrize("C", [2, 3, 10, 16, 17, 64, 100, 200, 256])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_curve_hist_small_classes_vs_aten_softmax(C, dtype):
    """Small-class row pass (C <= 256, T lanes per row, csrc/classification.hip mc_codes_small_kernel): the histogram
    equals the one built from ATen's softmax codes up to one-code moves of rounding-boundary quotients (same bound as
    the wide row pass), totals and the fused confusion matrix are exact."""
    N = 200_003  # not a multiple of the 64-row block
    g = torch.Generator(device="cuda").manual_seed(C)
    x = (torch.randn(N, C, device="cuda", generator=g) * 3).to(dtype)
    t = torch.randint(0, C, (N,), device="cuda", generator=g)
    t[::29] = -1
    hist = torch.zeros(C, 2, K.N_CODES, dtype=torch.long, device="cuda")
    cm = torch.zeros(C, C, dtype=torch.long, device="cuda")
    K.curve_hist_update(x, t, hist, "multiclass", -1, cm)
    keep = t != -1
    ref = torch.softmax(x[keep].float(), dim=1).to(dtype)
    href = _hist_from_scores(ref, t[keep], C)
    moved = int((hist - href).abs().sum()) // 2
    assert moved <= max(4, int((2e-5 if dtype == torch.bfloat16 else 1.5e-4) * N * C)), moved
    assert int(hist.sum()) == int(href.sum())
    cm_ref = torch.zeros(C, C, dtype=torch.long, device="cuda")
    cm_ref.view(-1).index_add_(0, t[keep] * C + x[keep].float().argmax(1), torch.ones_like(t[keep]))
    assert torch.equal(cm, cm_ref)


@pytest.mark.parametrize("C,n", [(4, 5000), (10, 5000), (64, 5000), (200, 5000), (4, 150_000), (10, 150_000)])
def test_curve_small_classes_speculation_and_rare_rows(C, n):
    """Module path through the small-class route: mode speculation flips (logits <-> probabilities, NaN batches),
    rare NaN / inf rows and ignore_index agree with the CPU implementation.  150k rows = more 64-row tiles than the
    FIXUP grid has blocks (the FIXUP pass must loop over tiles)."""
    import torchmetrics_forked_amd as tm

    batches = _flip_batches(C, n, seed=C)
    res = []
    for dev in ("cuda", "cpu"):
        m = tm.MulticlassAUROC(num_classes=C, average="macro", ignore_index=-1).to(dev)
        cmm = tm.MulticlassConfusionMatrix(num_classes=C, ignore_index=-1).to(dev)
        vals = []
        for x, t in batches:
            t = t.clone()
            t[::31] = -1
            m.update(x.to(dev), t.to(dev))
            cmm.update(x.to(dev), t.to(dev))
            vals.append(m.compute().item())
        res.append((vals, cmm.compute().cpu()))
    assert torch.equal(res[0][1], res[1][1])
    for a, b in zip(res[0][0], res[1][0]):
        assert abs(a - b) < 2e-5 or (a != a and b != b), (res[0][0], res[1][0])


def test_curve_scratch_cache_across_streams():
    """The two-pass route caches its class-major code scratch per (device, stream), at most 4 entries (LRU): metrics
    updated on six different streams (forcing evictions) give the same histograms as one update sequence on the
    default stream."""
    import torchmetrics_forked_amd as tm

    C, N = 1000, 4096
    g = torch.Generator().manual_seed(11)
    batches = [(torch.randn(N, C, generator=g).bfloat16().cuda(), torch.randint(0, C, (N,), generator=g).cuda()) for _ in range(6)]
    ref = tm.MulticlassAUROC(num_classes=C).cuda()
    for x, t in batches:
        ref.update(x, t)
    streams = [torch.cuda.Stream() for _ in range(6)]
    ms = [tm.MulticlassAUROC(num_classes=C).cuda() for _ in range(6)]
    torch.cuda.synchronize()
    for rnd in range(2):  # every metric sees every batch once, each round on another stream
        for k, (m, s) in enumerate(zip(ms, streams)):
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for x, t in batches[rnd * 3:(rnd + 1) * 3]:
                    m.update(x, t)
            torch.cuda.current_stream().wait_stream(s)
        streams = streams[1:] + streams[:1]
    torch.cuda.synchronize()
    want = ref.score_hist.cpu()
    for m in ms:
        assert torch.equal(m.score_hist.cpu(), want)


def test_calibration_error_deterministic_mode_reproducible():
    """Under torch.use_deterministic_algorithms(True) calibration error avoids its fp64-atomic kernels: two runs are
    bit-identical and equal the fast path to fp64 rounding."""
    import torchmetrics_forked_amd as tm

    g = torch.Generator().manual_seed(4)
    x = torch.randn(20000, 10, generator=g).softmax(1).cuda()
    t = torch.randint(0, 10, (20000,), generator=g).cuda()
    fast = tm.MulticlassCalibrationError(num_classes=10, n_bins=15).cuda()(x, t)
    # a host-resident metric takes the GPU batch (the reference keeps list states here): binned on the GPU, folded in
    host = tm.MulticlassCalibrationError(num_classes=10, n_bins=15)
    host.update(x, t)
    torch.testing.assert_close(host.compute(), fast.cpu(), rtol=1e-6, atol=1e-7)
    hb = tm.BinaryCalibrationError(n_bins=15)
    hb.update(x[:, 0], (t == 0).long())
    gb = tm.BinaryCalibrationError(n_bins=15).cuda()
    gb.update(x[:, 0], (t == 0).long())
    torch.testing.assert_close(hb.compute(), gb.compute().cpu(), rtol=1e-6, atol=1e-7)
    prev = torch.are_deterministic_algorithms_enabled()
    torch.use_deterministic_algorithms(True, warn_only=True)
    try:
        a = tm.MulticlassCalibrationError(num_classes=10, n_bins=15).cuda()(x, t)
        b = tm.MulticlassCalibrationError(num_classes=10, n_bins=15).cuda()(x, t)
    finally:
        torch.use_deterministic_algorithms(prev)
    assert torch.equal(a, b)
    torch.testing.assert_close(a, fast, rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("make", ["confmat", "auroc_binned", "collection"])
def test_host_state_metric_with_gpu_batch_raises_not_faults(make):
    """A metric whose tensor states stay on the host, fed GPU tensors: the device error of the reference (raised before
    any native kernel sees a host pointer), and the GPU keeps working."""
    import torchmetrics_forked_amd as tm

    x = torch.randn(256, 8).cuda()
    t = torch.randint(0, 8, (256,)).cuda()
    if make == "confmat":
        m = tm.MulticlassConfusionMatrix(num_classes=8)
    elif make == "auroc_binned":
        m = tm.MulticlassAUROC(num_classes=8, thresholds=5)
    else:
        m = tm.MetricCollection({"cm": tm.MulticlassConfusionMatrix(num_classes=8), "acc": tm.MulticlassAccuracy(num_classes=8)})
    with pytest.raises(RuntimeError, match="different devices|same device"):
        m.update(x, t)
    torch.cuda.synchronize()
    assert int(torch.ones(4, device="cuda").sum()) == 4
