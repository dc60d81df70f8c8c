"""Regression tests for the round-2 advisor findings."""
import pytest
import torch

import torchmetrics_forked_amd as tm
from torchmetrics_forked_amd.utilities.arena import StateArena
from torchmetrics_forked_amd.utilities.validation import DeferredChecks, host_checks
from torchmetrics_forked_amd.wrappers import BootStrapper


def test_catmetric_compute_does_not_alias_state():
    m = tm.CatMetric()
    m.update(torch.tensor([1.0, 2.0]))
    m.update(torch.tensor([3.0]))
    out = m.compute()
    out.mul_(0)  # a user editing the result must not reach the accumulated state
    m._computed = None
    torch.testing.assert_close(m.compute(), torch.tensor([1.0, 2.0, 3.0]))


def test_arena_clean_mark_lives_on_the_arena():
    a = StateArena([torch.ones(2), torch.ones(3)])
    a.clean = 2
    b = StateArena.adopt(a)
    assert b.clean == 2
    b.truncate(1)
    assert b.clean == 1
    b.append(torch.zeros(1))
    b.pop()
    assert b.clean == 0  # any other mutation forgets the mark
    assert StateArena().clean == 0


def test_catmetric_nan_drop_after_reset_starts_clean():
    m = tm.CatMetric(nan_strategy="ignore")
    m.update(torch.tensor([1.0, float("nan")]))
    assert m.compute().reshape(-1).tolist() == [1.0]
    m.reset()
    m.update(torch.tensor([float("nan"), 5.0]))
    m.update(torch.tensor([6.0]))
    assert m.compute().tolist() == [5.0, 6.0]


def test_deferred_flags_survive_an_aborted_compute_block():
    d = DeferredChecks()
    d.add(torch.tensor([True]), ValueError, "bad input")
    with pytest.raises(KeyError):
        with host_checks():
            d.check()
            raise KeyError("compute failed before the flags were read")
    with pytest.raises(ValueError, match="bad input"):
        d.check()  # the flag was put back: the invalid input still raises at the next compute


@pytest.mark.parametrize(
    "base, bad",
    [
        (lambda: tm.MulticlassAccuracy(num_classes=3), (torch.tensor([0, 1, 2, 1]), torch.tensor([0, 5, 1, 2]))),
        (lambda: tm.MeanSquaredError(), (torch.rand(4), torch.rand(5))),
    ],
)
def test_bootstrapper_weighted_path_still_validates(base, bad):
    bs = BootStrapper(base(), num_bootstraps=4)
    with pytest.raises((RuntimeError, ValueError)):
        bs.update(*bad)


def test_bootstrapper_weighted_path_updates_in_place():
    bs = BootStrapper(tm.MeanSquaredError(), num_bootstraps=3, sampling_strategy="multinomial")
    ptrs = [m.sum_squared_error.data_ptr() for m in bs.metrics]
    bs.update(torch.rand(16), torch.rand(16))
    assert [m.sum_squared_error.data_ptr() for m in bs.metrics] == ptrs
    assert all(int(m.total) == 16 for m in bs.metrics)


def test_use_native_rejects_mixed_devices_before_launch():
    """ops.use_native(t, *others): a host tensor mixed with a GPU tensor raises torch's device error (checked on the
    host, before any native launch could receive a host pointer); all-host calls stay on the CPU path."""
    import pytest
    import torch

    from torchmetrics_forked_amd import ops

    a = torch.zeros(3)
    assert ops.use_native(a, torch.zeros(2), None, torch.tensor(1.0)) is False  # host-only: the CPU path
    err = ops._device_error(torch.device("cuda", 0), torch.device("cpu"))
    assert "same device" in str(err)  # the message the Metric wrapper re-words (GPU cases: tests/test_ops_gpu.py)
