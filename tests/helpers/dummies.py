"""Small metrics used by the core-runtime tests (module level so they pickle into DDP workers)."""
import torch
from torch import Tensor

from torchmetrics_forked_amd.metric import Metric
from torchmetrics_forked_amd.utilities.data import dim_zero_cat


class DummySum(Metric):
    full_state_update = False

    def __init__(self, **kw):
        super().__init__(**kw)
        self.add_state("x", torch.tensor(0.0), dist_reduce_fx="sum")

    def update(self, v):
        self.x += v

    def compute(self):
        return self.x


class DummyCat(Metric):
    full_state_update = False

    def __init__(self, **kw):
        super().__init__(**kw)
        self.add_state("x", [], dist_reduce_fx="cat")

    def update(self, v):
        self.x.append(torch.as_tensor(v).reshape(-1).float())

    def compute(self):
        return dim_zero_cat(self.x)


class DummyList(Metric):
    """``None``-reduced list state (gathered, rank-interleaved)."""

    full_state_update = True

    def __init__(self, **kw):
        super().__init__(**kw)
        self.add_state("x", [], dist_reduce_fx=None)

    def update(self, v):
        self.x.append(torch.as_tensor(v).float())

    def compute(self):
        return self.x


class DummyMinMaxMean(Metric):
    full_state_update = False

    def __init__(self, **kw):
        super().__init__(**kw)
        self.add_state("mn", torch.tensor(float("inf")), dist_reduce_fx="min")
        self.add_state("mx", torch.tensor(-float("inf")), dist_reduce_fx="max")
        self.add_state("mean", torch.tensor(0.0), dist_reduce_fx="mean")
        self.add_state("custom", torch.zeros(3), dist_reduce_fx=lambda s: s.prod(0))

    def update(self, v):
        v = torch.as_tensor(v, dtype=torch.float32)
        self.mn = torch.min(self.mn, v.min())
        self.mx = torch.max(self.mx, v.max())
        self.mean = v.mean()
        self.custom = torch.full((3,), float(v.sum()))

    def compute(self):
        return self.mn, self.mx, self.mean


class DummyStacked(Metric):
    """``None``-reduced tensor state: synced value is stacked ``(world, ...)``."""

    full_state_update = True

    def __init__(self, **kw):
        super().__init__(**kw)
        self.add_state("stacked", torch.zeros(2), dist_reduce_fx=None)

    def update(self, v):
        v = torch.as_tensor(v, dtype=torch.float32)
        self.stacked = torch.stack([v.min(), v.max()])

    def compute(self):
        return self.stacked
