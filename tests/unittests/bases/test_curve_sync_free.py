"""Host-synchronisation-free curve sync (``_CurveMetric._sync_dist_free``, round 6).

The default histogram sync reads a gathered per-rank summary on the host to size its collectives (int32 narrowing,
occupied code range).  Under HIP-graph capture, or with ``TMX_CURVE_SYNC_FREE=1``, the histogram travels over its
full code range as int64 and the per-class code ranges are combined on the device instead: no device-to-host read.
Checked here: identical results to the default sync on 2 gloo ranks (replicated and class-sharded, a rank without
a batch, disjoint code ranges), the replicated default sync reusing its expanded-histogram buffer, and on the GPU a
``compute()`` with the sync under ``torch.cuda.set_sync_debug_mode("error")``.
"""
import pytest
import torch

from tests.helpers.multirank import run_multirank


def _batches(world, C=5, seed=3):
    g = torch.Generator().manual_seed(seed)
    out = []
    for r in range(world):
        lo = 0.6 * r / max(1, world - 1)
        p = (lo + torch.rand(48, C, generator=g) * 0.4).bfloat16()
        out.append((p, torch.randint(0, C, (48,), generator=g)))
    return out


def _sync_free_worker(rank, world, device):
    from torchmetrics_forked_amd.classification import MulticlassAUROC, MulticlassAveragePrecision, MulticlassROC
    from torchmetrics_forked_amd.classification import precision_recall_curve as prc

    batches = _batches(world)
    calls = []
    orig = prc._CurveMetric._sync_dist_free
    prc._CurveMetric._sync_dist_free = lambda self, group: (calls.append(1), orig(self, group))[1]
    for cls in (MulticlassAUROC, MulticlassAveragePrecision, MulticlassROC):
        for sharded in (False, True):
            if cls is MulticlassROC and sharded:
                continue
            for empty_rank in (None, 1):
                kw = {"num_classes": 5}
                if cls is not MulticlassROC:
                    kw.update(average="none", sharded_compute=sharded)
                ref, free = cls(**kw).to(device), cls(**kw).to(device)
                if rank != empty_rank:
                    p, t = batches[rank]
                    for m in (ref, free):
                        m.update(p.to(device), t.to(device))
                prc._SYNC_FREE = False
                a = ref.compute()
                prc._SYNC_FREE = True
                try:
                    b = free.compute()
                finally:
                    prc._SYNC_FREE = False
                if isinstance(a, tuple):
                    for x, y in zip(a, b):
                        for u, v in zip(x, y):
                            assert torch.equal(u, v)
                else:
                    torch.testing.assert_close(a, b, rtol=0, atol=1e-7, equal_nan=True)
                # the local state is back after the sync
                if rank != empty_rank:
                    assert free.score_hist.shape == (5, 2, 16384)
    prc._CurveMetric._sync_dist_free = orig
    assert len(calls) == 10, len(calls)


def test_sync_free_matches_default_sync():
    run_multirank(_sync_free_worker, 2)


def _replicated_buffer_worker(rank, world, device):
    from torchmetrics_forked_amd.classification import MulticlassAUROC

    g = torch.Generator().manual_seed(9 + rank)
    m = MulticlassAUROC(num_classes=4, average="none")
    ref = MulticlassAUROC(num_classes=4, average="none")
    ptrs = []
    for lo, width in ((0.9, 0.1), (0.0, 0.05), (0.0, 1.0)):
        m.reset()
        ref.reset()
        p = (lo + torch.rand(32, 4, generator=g) * width).bfloat16()
        t = torch.randint(0, 4, (32,), generator=g)
        m.update(p, t)
        ps = [torch.zeros_like(p) for _ in range(world)]
        ts = [torch.zeros_like(t) for _ in range(world)]
        torch.distributed.all_gather(ps, p)
        torch.distributed.all_gather(ts, t)
        for pp, tt in zip(ps, ts):
            ref.update(pp, tt)
        ref.sync_on_compute = False
        torch.testing.assert_close(m.compute(), ref.compute(), rtol=0, atol=1e-7, equal_nan=True)
        ptrs.append(m.__dict__["_synced_buf"][0].data_ptr())
    assert len(set(ptrs)) == 1


def test_replicated_sync_reuses_expanded_buffer():
    run_multirank(_replicated_buffer_worker, 2)


def _sync_debug_worker(rank, world, device):
    """One-rank RCCL group on the GPU: the sync-free sync issues its collectives without any device-to-host read
    (torch's sync debug mode raises on one); compute() with it gives the unsynced metric's value."""
    from torchmetrics_forked_amd.classification import MulticlassAUROC
    from torchmetrics_forked_amd.classification import precision_recall_curve as prc

    g = torch.Generator(device=device).manual_seed(1)
    for sharded in (False, True):
        m = MulticlassAUROC(num_classes=10, average="macro", sharded_compute=sharded).to(device)
        ref = MulticlassAUROC(num_classes=10, average="macro").to(device)
        x = torch.randn(4096, 10, device=device, generator=g).bfloat16()
        t = torch.randint(0, 10, (4096,), device=device, generator=g)
        m.update(x, t)
        ref.update(x, t)
        ref.sync_on_compute = False
        expect = ref.compute()
        local = m.score_hist.clone()
        torch.cuda.synchronize()
        prc._SYNC_FREE = True
        try:
            torch.cuda.set_sync_debug_mode("error")
            try:
                m.sync()
                synced = m.score_hist.clone()
                m.unsync()
            finally:
                torch.cuda.set_sync_debug_mode("default")
            got = m.compute()
        finally:
            prc._SYNC_FREE = False
        assert torch.equal(m.score_hist, local)
        assert torch.equal(synced, local if not sharded else local[: synced.shape[0]])
        torch.testing.assert_close(got, expect, rtol=0, atol=1e-7)


@pytest.mark.gpu
def test_sync_free_has_no_host_sync_on_gpu():
    run_multirank(_sync_debug_worker, 1, backend="nccl")
