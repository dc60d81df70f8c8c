"""Metric-state synchronisation at world sizes >= 2 on the production backend (nccl = RCCL over xGMI on MI355X)
and, with the very same check bodies, on gloo (CPU, runs in the default suite).

What is checked on every rank (reference semantics: ``/root/reference/src/torchmetrics/metric.py:423-453``,
``/root/reference/src/torchmetrics/utilities/distributed.py:97-147``):

* coalesced all-reduce buckets for ``sum`` / ``mean`` / ``max`` / ``min`` states over several dtypes;
* ``cat`` lists of uneven length and shape per rank, a rank with no element, ``None``-reduced lists
  (element-major, rank-interleaved) and ``None``-reduced tensors (stacked);
* class-sharded AUROC / AP (reduce-scatter of the exact histogram by class) equal to the replicated computation
  and to a single-process computation over every rank's data;
* the int32 narrowing of histogram collectives: exact int64 sums also when a bin exceeds int32;
* a MetricCollection (fused AUROC + confusion matrix + accuracy) against the single-process result;
* async sync handles; mismatched score dtypes across ranks raise on every rank (no hang);
* a rank that never joins surfaces as ``SyncTimeoutError`` (gloo only: a timed-out RCCL collective aborts the
  communicator, which is the intended production behaviour but would end the test group).

The RCCL variants need >= 2 visible GPUs (one process per GPU) and skip otherwise.
"""
import pytest
import torch

from tests.helpers.multirank import run_multirank


def _data(r: int, n: int = 96, c: int = 37, dtype=torch.bfloat16):
    g = torch.Generator().manual_seed(1000 + r)
    x = torch.randn(n + 7 * r, c, generator=g)
    t = torch.randint(0, c, (n + 7 * r,), generator=g)
    return x.to(dtype), t


def check_reductions(rank, world, device):
    from tests.helpers.dummies import DummyMinMaxMean, DummySum
    from torchmetrics_forked_amd.aggregation import MaxMetric, MeanMetric, MinMetric, SumMetric

    m = DummySum().to(device)
    m.update(torch.tensor(float(rank + 1), device=device))
    assert float(m.compute()) == world * (world + 1) / 2
    mm = DummyMinMaxMean().to(device)
    mm.update(torch.tensor([rank * 1.0, rank + 3.0], device=device))
    mm.sync()
    assert float(mm.mn) == 0.0 and float(mm.mx) == world + 2.0
    mm.unsync()
    vals = [torch.arange(5, dtype=torch.float64) * (r + 1) for r in range(world)]
    allv = torch.cat(vals)
    for cls, expect in ((SumMetric, allv.sum()), (MeanMetric, allv.mean()), (MaxMetric, allv.max()), (MinMetric, allv.min())):
        met = cls().to(device)
        met.update(vals[rank].to(device))
        got = met.compute()
        assert torch.allclose(got.double().cpu(), expect, rtol=1e-6), (cls.__name__, got, expect)
    # integer / bool / half states in one bucketed call
    from torchmetrics_forked_amd.parallel.sync import sync_states
    from torchmetrics_forked_amd.utilities.data import dim_zero_max, dim_zero_sum

    states = {
        "a": torch.full((3,), rank + 1, dtype=torch.int32, device=device),
        "b": torch.full((2, 2), rank + 1, dtype=torch.int64, device=device),
        "c": torch.tensor([rank % 2 == 0, True], device=device),
        "d": torch.full((4,), 0.5 * (rank + 1), dtype=torch.bfloat16, device=device),
    }
    out = sync_states(states, {"a": dim_zero_sum, "b": dim_zero_sum, "c": dim_zero_sum, "d": dim_zero_max})
    s = world * (world + 1) // 2
    assert out["a"].dtype == torch.int32 and out["a"].tolist() == [s] * 3
    assert out["b"].tolist() == [[s, s], [s, s]]
    assert out["c"].tolist() == [True, True]
    assert out["d"].dtype == torch.bfloat16 and float(out["d"][0]) == 0.5 * world


def check_lists(rank, world, device):
    from tests.helpers.dummies import DummyCat, DummyList, DummyStacked

    m = DummyCat().to(device)
    for i in range(rank + 1):  # rank r holds r + 1 elements of length i + 1
        m.update(torch.arange(i + 1, device=device).float() + 100 * rank)
    got = m.compute().cpu().tolist()
    exp = [float(j + 100 * r) for r in range(world) for i in range(r + 1) for j in range(i + 1)]
    assert got == exp, (got, exp)
    e = DummyCat().to(device)
    if rank == world - 1:
        e.update(torch.tensor([5.0, 6.0], device=device))
    else:
        e._update_count = 1
    assert e.compute().cpu().tolist() == [5.0, 6.0]
    li = DummyList().to(device)
    for k in range(1 + (rank % 2)):  # uneven list lengths
        li.update(torch.tensor(rank * 10.0 + k, device=device))
    out = [float(t) for t in li.compute()]
    exp = [r * 10.0 + k for k in range(2) for r in range(world) if k < 1 + (r % 2)]
    assert out == exp, (out, exp)
    st = DummyStacked().to(device)
    st.update(torch.tensor([rank * 1.0, rank + 3.0], device=device))
    assert tuple(st.compute().shape) == (world, 2)


def check_sharded_auroc(rank, world, device):
    from torchmetrics_forked_amd.classification import MulticlassAUROC, MulticlassAveragePrecision

    c = 37
    for cls in (MulticlassAUROC, MulticlassAveragePrecision):
        for average in ("macro", "weighted", "none"):
            sharded = cls(num_classes=c, average=average, sharded_compute=True).to(device)
            plain = cls(num_classes=c, average=average).to(device)
            single = cls(num_classes=c, average=average, sync_on_compute=False).to(device)
            for step in range(2):
                x, t = _data(rank + world * step, c=c)
                sharded.update(x.to(device), t.to(device))
                plain.update(x.to(device), t.to(device))
                for r in range(world):
                    xr, tr = _data(r + world * step, c=c)
                    single.update(xr.to(device), tr.to(device))
            a, b, ref = sharded.compute(), plain.compute(), single.compute()
            assert torch.allclose(a.cpu(), ref.cpu(), atol=1e-6, equal_nan=True), (cls.__name__, average, a, ref)
            assert torch.allclose(b.cpu(), ref.cpu(), atol=1e-6, equal_nan=True), (cls.__name__, average, b, ref)
            assert sharded.score_hist.shape[0] == c  # local state restored


def check_narrowing(rank, world, device):
    from torchmetrics_forked_amd.classification import MulticlassAUROC

    for big in (False, True):
        for sharded in (False, True):
            m = MulticlassAUROC(num_classes=3, sharded_compute=sharded).to(device)
            m.update(torch.randn(16, 3).softmax(-1).bfloat16().to(device), torch.randint(0, 3, (16,)).to(device))
            if big:
                m.score_hist[:, 0, 5] += 2**31 - 10
                m._invalidate_range()
            local = m.score_hist.clone()
            parts = torch.empty(world, *local.shape, dtype=local.dtype, device=local.device)
            torch.distributed.all_gather_into_tensor(parts.view(-1), local.reshape(-1))
            expect = parts.sum(0)
            m.sync()
            got = m.score_hist
            if sharded:
                first, owned, _, _ = m._shard_info
                expect = expect[first : first + owned]
            assert got.dtype == torch.long and torch.equal(got, expect)
            m.unsync()
            assert torch.equal(m.score_hist, local)


def check_collection(rank, world, device):
    import torchmetrics_forked_amd as tm

    c = 37

    def coll(**kw):
        return tm.MetricCollection({
            "auroc": tm.MulticlassAUROC(num_classes=c, **kw),
            "cm": tm.MulticlassConfusionMatrix(num_classes=c, **{k: v for k, v in kw.items() if k != "sharded_compute"}),
            "acc": tm.MulticlassAccuracy(num_classes=c, **{k: v for k, v in kw.items() if k != "sharded_compute"}),
        }).to(device)

    dist_c = coll(sharded_compute=True)
    single = coll(sync_on_compute=False)
    for step in range(3):
        x, t = _data(rank + world * step, c=c)
        dist_c.update(x.to(device), t.to(device))
        for r in range(world):
            xr, tr = _data(r + world * step, c=c)
            single.update(xr.to(device), tr.to(device))
    a, b = dist_c.compute(), single.compute()
    for k in a:
        assert torch.allclose(a[k].double().cpu(), b[k].double().cpu(), atol=1e-6), (k, a[k], b[k])


def check_async(rank, world, device):
    from torchmetrics_forked_amd.aggregation import CatMetric, MaxMetric, SumMetric

    ms = [SumMetric().to(device), MaxMetric().to(device), CatMetric().to(device)]
    for m in ms:
        m.update(torch.arange(3, dtype=torch.float32, device=device) + 10 * rank)
    handles = [m.sync(async_op=True) for m in ms]
    _ = torch.randn(64, 64, device=device) @ torch.randn(64, 64, device=device)
    for h in handles:
        h.wait()
    assert float(ms[0].sum_value) == sum(3.0 + 30 * r for r in range(world))
    assert float(ms[1].max_value) == 10 * (world - 1) + 2
    vals = ms[2].value if isinstance(ms[2].value, torch.Tensor) else torch.cat(list(ms[2].value))
    assert vals.numel() == 3 * world
    for m in ms:
        m.unsync()


def check_dtype_mismatch(rank, world, device):
    from torchmetrics_forked_amd.classification import MulticlassAUROC

    m = MulticlassAUROC(num_classes=5).to(device)
    x = torch.randn(32, 5).softmax(-1)
    m.update(x.to(torch.bfloat16 if rank == 0 else torch.float16).to(device), torch.randint(0, 5, (32,)).to(device))
    with pytest.raises(RuntimeError, match="different 16-bit dtypes"):
        m.compute()
    # an empty rank adopts the others' dtype
    e = MulticlassAUROC(num_classes=5).to(device)
    if rank == 0:
        e.update(x.half().to(device), torch.randint(0, 5, (32,)).to(device))
    else:
        e._update_count = 1
    e.sync()
    assert e._hist_dtype == torch.float16
    e.unsync()


def check_sharded_retrieval(rank, world, device):
    """Query-sharded retrieval (all_to_all of rows to the owning rank) equals the replicated computation and the
    single-process computation over every rank's rows in rank order; the last rank holds no rows at all."""
    import torchmetrics_forked_amd as tm

    def rows(r):
        g = torch.Generator().manual_seed(77 + r)
        n = 0 if (r == world - 1 and world > 2) else 40 + 9 * r
        idx = torch.randint(0, 11, (n,), generator=g)
        preds = (torch.rand(n, generator=g) * 8).floor() / 8  # ties inside queries
        target = (torch.rand(n, generator=g) < 0.3).long()
        target[idx == 3] = 0  # query 3 has no positive document
        return idx, preds, target

    makers = [
        lambda **kw: tm.RetrievalMAP(empty_target_action="skip", **kw),
        lambda **kw: tm.RetrievalMRR(empty_target_action="pos", **kw),
        lambda **kw: tm.RetrievalNormalizedDCG(top_k=3, **kw),
        lambda **kw: tm.RetrievalPrecision(top_k=2, adaptive_k=True, **kw),
        lambda **kw: tm.RetrievalPrecisionRecallCurve(**kw),
        lambda **kw: tm.RetrievalFallOut(**kw),
    ]
    idx, preds, target = rows(rank)
    all_rows = [rows(r) for r in range(world)]
    for make in makers:
        sharded, replicated, single = make(sharded_compute=True).to(device), make().to(device), make(sync_on_compute=False)
        if idx.numel():
            sharded.update(preds.to(device), target.to(device), indexes=idx.to(device))
            replicated.update(preds.to(device), target.to(device), indexes=idx.to(device))
        for i, p, t in all_rows:
            if i.numel():
                single.update(p, t, indexes=i)
        a, b = sharded.compute(), replicated.compute()
        c = single.compute()
        a, b = (a if isinstance(a, tuple) else (a,)), (b if isinstance(b, tuple) else (b,))
        c = c if isinstance(c, tuple) else (c,)
        for x, y, z in zip(a, b, c):
            torch.testing.assert_close(x.cpu().double(), y.cpu().double(), atol=1e-6, rtol=0)
            torch.testing.assert_close(x.cpu().double(), z.double(), atol=1e-6, rtol=0)
        # the local state is restored after compute (unsync)
        assert sum(t.numel() for t in sharded.indexes) == idx.numel()
    # "error" policy raises on every rank when any rank owns an empty query
    err = tm.RetrievalMAP(empty_target_action="error", sharded_compute=True).to(device)
    if idx.numel():
        err.update(preds.to(device), target.to(device), indexes=idx.to(device))
    with pytest.raises(ValueError, match="no positive target"):
        err.compute()


def check_sharded_map(rank, world, device):
    """Class-sharded MeanAveragePrecision (rows routed by class with all_to_all, MAX all-reduce of the tables) equals
    the replicated computation and the single-process computation over every rank's images in rank order."""
    from torchmetrics_forked_amd.detection import MeanAveragePrecision

    def images(r):
        g = torch.Generator().manual_seed(500 + r)
        out_p, out_t = [], []
        for _ in range(3 + r):
            ng = int(torch.randint(1, 6, (1,), generator=g))
            xy = torch.rand(ng, 2, generator=g) * 300
            gt = torch.cat([xy, xy + torch.rand(ng, 2, generator=g) * 120 + 4], 1)
            gl = torch.randint(0, 6, (ng,), generator=g) * 2 + 1
            det = torch.cat([gt + torch.randn(ng, 4, generator=g) * 6, gt[:2] + 40])
            det[:, 2:] = torch.maximum(det[:, 2:], det[:, :2] + 1)
            dl = torch.cat([gl, torch.randint(0, 6, (det.shape[0] - ng,), generator=g) * 2 + 1])
            out_p.append({"boxes": det, "scores": (torch.rand(det.shape[0], generator=g) * 10).floor() / 10, "labels": dl})
            out_t.append({"boxes": gt, "labels": gl, "iscrowd": (torch.rand(ng, generator=g) < 0.2).long()})
        return out_p, out_t

    to = lambda lst: [{k: v.to(device) for k, v in d.items()} for d in lst]  # noqa: E731
    sharded = MeanAveragePrecision(class_metrics=True, sharded_compute=True).to(device)
    replicated = MeanAveragePrecision(class_metrics=True).to(device)
    single = MeanAveragePrecision(class_metrics=True, sync_on_compute=False)
    p, t = images(rank)
    sharded.update(to(p), to(t))
    replicated.update(to(p), to(t))
    per_rank = [images(r) for r in range(world)]
    for e in range(max(len(x[0]) for x in per_rank)):  # the gather's element-major, rank-interleaved image order
        for pr, tr in per_rank:
            if e < len(pr):
                single.update([pr[e]], [tr[e]])
    a, b, c = sharded.compute(), replicated.compute(), single.compute()
    for k in c:
        torch.testing.assert_close(a[k].cpu(), b[k].cpu(), atol=0, rtol=0, msg=k)
        torch.testing.assert_close(a[k].cpu(), c[k], atol=0, rtol=0, msg=k)


def check_timeout(rank, world, device):
    import time

    from torchmetrics_forked_amd.aggregation import SumMetric
    from torchmetrics_forked_amd.parallel import SyncTimeoutError

    m = SumMetric(sync_timeout=1.5)
    m.update(torch.tensor(float(rank + 1)))
    if rank == 0:
        with pytest.raises(SyncTimeoutError, match=f"rank 0 of {world}"):
            m.compute()
    else:
        time.sleep(4.0)
        assert float(m.compute()) == world * (world + 1) / 2
    torch.distributed.barrier()
    # async path honours the metric's bound too
    a = SumMetric(sync_timeout=1.5)
    a.update(torch.tensor(1.0))
    if rank == 0:
        h = a.sync(async_op=True)
        with pytest.raises(SyncTimeoutError):
            h.wait()
    else:
        time.sleep(4.0)
        a.sync()
        a.unsync()
    torch.distributed.barrier()


CHECKS = [check_reductions, check_lists, check_sharded_auroc, check_narrowing, check_collection, check_async,
          check_dtype_mismatch, check_sharded_retrieval, check_sharded_map]


def _run_all(rank, world, device):
    for fn in CHECKS:
        fn(rank, world, device)
        torch.distributed.barrier()


@pytest.mark.parametrize("world", [2, 3])
def test_multirank_gloo(world):
    run_multirank(_run_all, world, "gloo")


def test_multirank_gloo_timeout():
    run_multirank(check_timeout, 2, "gloo")


def _gpus() -> int:
    return torch.cuda.device_count() if torch.cuda.is_available() else 0


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 0])
def test_multirank_rccl(world):
    n = _gpus()
    world = world or n
    if n < 2 or world > n:
        pytest.skip(f"needs {max(world, 2)} GPUs (one RCCL rank per GPU), found {n}")
    run_multirank(_run_all, min(world, 8), "nccl", timeout=300)


def _run_sharded(rank, world, device):
    check_sharded_retrieval(rank, world, device)
    torch.distributed.barrier()
    check_sharded_map(rank, world, device)


@pytest.mark.gpu
def test_sharded_compute_gpu_states_gloo():
    """Sharded retrieval / mAP with GPU-resident states (device evaluator, GPU Grouped) on a one-GPU box: two ranks
    share cuda:0 and exchange over gloo."""
    if _gpus() < 1:
        pytest.skip("needs a GPU")
    run_multirank(_run_sharded, 2, "gloo_cuda", timeout=300)

