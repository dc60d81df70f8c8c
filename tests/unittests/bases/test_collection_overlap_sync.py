"""MetricCollection.compute: grouped async syncs (all-reduces enqueued up front, each group waited for when its first
member computes) give the same results as each member syncing on its own (gloo, world size 2)."""
import torch

from tests.helpers.multirank import run_multirank


def check_overlapped_collection(rank: int, world: int, device: torch.device) -> None:
    import torchmetrics_forked_amd as tm
    from torchmetrics_forked_amd.parallel import sync as sync_mod

    C = 600  # the confusion matrix alone (600 x 600 int64 = 2.9 MB) fills an overlap group
    make = lambda: {  # noqa: E731
        "cm": tm.MulticlassConfusionMatrix(num_classes=C),
        "acc": tm.MulticlassAccuracy(num_classes=C),
        "f1": tm.MulticlassF1Score(num_classes=C, average="macro"),
        "cat": tm.CatMetric(),
        "mse": tm.MeanSquaredError(),
    }
    coll = tm.MetricCollection(make(), compute_groups=False)
    solo = make()
    g = torch.Generator().manual_seed(7 + rank)
    for step in range(3):
        p = torch.randn(64 + 8 * rank, C, generator=g)
        t = torch.randint(0, C, (64 + 8 * rank,), generator=g)
        v = torch.randn(5 + rank + step, generator=g)
        coll["cm"].update(p, t)
        coll["acc"].update(p, t)
        coll["f1"].update(p, t)
        coll["cat"].update(v)
        coll["mse"].update(v, v * 0.5)
        solo["cm"].update(p, t)
        solo["acc"].update(p, t)
        solo["f1"].update(p, t)
        solo["cat"].update(v)
        solo["mse"].update(v, v * 0.5)
    starts = []
    orig = sync_mod.PendingSyncMany.__init__

    def spy(self, *a, **k):  # noqa: ANN001
        starts.append(len(a[0]))
        orig(self, *a, **k)

    sync_mod.PendingSyncMany.__init__ = spy
    try:
        out = coll.compute()
    finally:
        sync_mod.PendingSyncMany.__init__ = orig
    assert len(starts) >= 2, starts  # the big confusion matrix closes its own group
    for k, m in solo.items():
        ref = m.compute()
        torch.testing.assert_close(out[k], ref)
    # local states are back after compute (accumulation continues)
    assert not any(m._is_synced for m in coll.values(copy_state=False))
    assert int(coll["cm"].confmat.sum()) == 3 * (64 + 8 * rank)


def test_collection_overlapped_sync_gloo2():
    run_multirank(check_overlapped_collection, 2, "gloo")
